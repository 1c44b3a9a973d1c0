"""generate_test (example_gen.rs:11-64) with the reference RNG stack
(rand 0.8 StdRng = ChaCha12, seed_from_u64). `seed` generalises the
reference's hardcoded seed 0. Host-side input generation (not the hot path)."""
import ctypes

from . import _lib


def generate_test(alphabet_size, seq_len, num_samples, error_rate, seed=0):
    """Returns (consensus bytes, list of sample bytes)."""
    L = _lib.lib()
    h = ctypes.c_void_p()
    rc = L.wc_generate_test(int(alphabet_size), int(seq_len), int(num_samples), float(error_rate), int(seed),
                            ctypes.byref(h))
    if rc != _lib.WC_OK:
        raise _lib.WaffleConError("generate_test: invalid arguments", rc)
    try:
        n = ctypes.c_uint64()
        p = L.wc_gen_consensus(h, ctypes.byref(n))
        con = ctypes.string_at(p, n.value) if n.value else b""
        samples = []
        for i in range(num_samples):
            p = L.wc_gen_sample(h, i, ctypes.byref(n))
            samples.append(ctypes.string_at(p, n.value) if n.value else b"")
        return con, samples
    finally:
        L.wc_gen_free(h)
