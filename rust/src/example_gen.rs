//! example_gen.rs:11-64: generate_test with the reference's RNG
//! (StdRng::seed_from_u64(0)), restated in the library (wc_generate_test).
use crate::ffi;

/// example_gen.rs:11
pub fn generate_test(alphabet_size: u8, seq_len: usize, num_samples: usize, error_rate: f64) -> (Vec<u8>, Vec<Vec<u8>>) {
    generate_test_seeded(alphabet_size, seq_len, num_samples, error_rate, 0)
}

/// The same with another seed (the reference hardcodes 0; the bench loci use the locus id)
pub fn generate_test_seeded(alphabet_size: u8, seq_len: usize, num_samples: usize, error_rate: f64,
                            seed: u64) -> (Vec<u8>, Vec<Vec<u8>>) {
    unsafe {
        let mut g = std::ptr::null_mut();
        let rc = ffi::wc_generate_test(alphabet_size, seq_len as u64, num_samples as u64, error_rate, seed, &mut g);
        assert_eq!(rc, ffi::WC_OK, "wc_generate_test failed");
        let mut n = 0u64;
        let c = ffi::wc_gen_consensus(g, &mut n);
        let consensus = std::slice::from_raw_parts(c, n as usize).to_vec();
        let samples = (0..num_samples as u64)
            .map(|i| {
                let s = ffi::wc_gen_sample(g, i, &mut n);
                std::slice::from_raw_parts(s, n as usize).to_vec()
            })
            .collect();
        ffi::wc_gen_free(g);
        (consensus, samples)
    }
}
