"""GPU parity of the 2-bit packed batch upload (host.cpp
pack_read_*, pack2.hip): a batch whose reads are raw codes 0..3 or ASCII
A/C/G/T crosses PCIe at 2 bits per base and is expanded on the device. The
expanded arena must give the same consensuses and work counters as the byte
upload (WC_PACK=0) and the oracle; a batch with one byte outside the alphabet
must fall back to the byte path (wc_last_upload_packed = 0). WC_PACK=1 forces
packing below its default 16 MiB threshold so small batches exercise it."""
import pytest

import oracle_ffi as orc

pytestmark = pytest.mark.gpu

hip = pytest.importorskip("hip_runner")

KEYS = ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored", "nodes_ignored",
        "peak_queue_size", "row_bytes")
ACGT = bytes.maketrans(bytes(range(4)), b"ACGT")


def _problems(ascii_, n=12):
    import waffle_con_amd as w
    out = []
    for i in range(n):
        # ragged: read lengths not multiples of 4 or 16
        reads = w.generate_test(4, 301 + 37 * i, 6 + i % 5, 0.02, 500 + i)[1]
        if ascii_:
            reads = [r.translate(ACGT) for r in reads]
        out.append(reads)
    return out


def _run(problems, monkeypatch, pack):
    from waffle_con_amd import _lib
    monkeypatch.setenv("WC_PACK", pack)
    got, stats = hip.consensus_batch(problems, counters=True, min_count=2)
    return got, stats, _lib.default_context().last_upload_packed()


@pytest.mark.parametrize("scalar", [False, True])
@pytest.mark.parametrize("ascii_", [False, True])
def test_packed_upload_matches_byte_upload(ascii_, scalar, monkeypatch):
    if scalar:  # the packer without AVX-512 (WC_PACK_SCALAR test hook)
        monkeypatch.setenv("WC_PACK_SCALAR", "1")
    probs = _problems(ascii_)
    got_p, st_p, packed = _run(probs, monkeypatch, "1")
    got_b, st_b, unpacked = _run(probs, monkeypatch, "0")
    total = sum((len(r) + 15) // 16 * 16 for p in probs for r in p)
    assert packed == total // 4
    assert unpacked == 0
    assert got_p == got_b
    for k in KEYS:
        assert st_p[k] == st_b[k], k
    for p, g in zip(probs[:4], got_p[:4]):
        assert g == orc.consensus(p, min_count=2)


def test_packed_upload_falls_back_outside_alphabet(monkeypatch):
    probs = _problems(True, n=4)
    probs[3] = list(probs[3])
    r = bytearray(probs[3][-1])
    r[len(r) // 2] = ord("N")
    probs[3][-1] = bytes(r)
    got, _, packed = _run(probs, monkeypatch, "1")
    assert packed == 0
    for p, g in zip(probs, got):
        assert g == orc.consensus(p, min_count=2)


@pytest.mark.parametrize("bad_last", [False, True])
def test_packed_upload_several_chunks_and_threads(bad_last, monkeypatch):
    """The production shape on a small batch: eight chunks, each packed by
    several threads while the previous chunks' copies are in flight
    (WC_UPLOAD_CHUNK_SHIFT / WC_UPLOAD_THREAD_SHIFT shrink the 64 MiB chunks
    and 8 MiB per thread). With a byte outside the alphabet in the batch's
    last read, the packed copies already queued are dropped and the batch
    goes the byte way."""
    monkeypatch.setenv("WC_UPLOAD_CHUNK_SHIFT", "12")
    monkeypatch.setenv("WC_UPLOAD_THREAD_SHIFT", "9")
    probs = _problems(True, n=16)
    if bad_last:
        probs[-1] = list(probs[-1])
        r = bytearray(probs[-1][-1])
        r[-1] = ord("N")
        probs[-1][-1] = bytes(r)
    total = sum((len(r) + 15) // 16 * 16 for p in probs for r in p)
    assert total >> 12 >= 8  # eight chunks
    got_p, st_p, packed = _run(probs, monkeypatch, "1")
    got_b, st_b, _ = _run(probs, monkeypatch, "0")
    assert packed == (0 if bad_last else total // 4)
    assert got_p == got_b
    for k in KEYS:
        assert st_p[k] == st_b[k], k
    for p, g in zip(probs[-3:], got_p[-3:]):
        assert g == orc.consensus(p, min_count=2)
