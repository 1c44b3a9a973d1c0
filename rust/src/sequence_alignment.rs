//! sequence_alignment.rs:18-87: pairwise WFA edit distance (host reference
//! API of the library; device::wfa_ed_batch runs many pairs on the GPU).
use crate::ffi;

/// sequence_alignment.rs:18: end-to-end edit distance with '*' as wildcard
pub fn wfa_ed(v1: &[u8], v2: &[u8]) -> usize {
    wfa_ed_config(v1, v2, true, Some(b'*'))
}

/// sequence_alignment.rs:36
pub fn wfa_ed_config(v1: &[u8], v2: &[u8], require_both_end: bool, wildcard: Option<u8>) -> usize {
    unsafe {
        ffi::wc_wfa_ed_config(v1.as_ptr(), v1.len() as u64, v2.as_ptr(), v2.len() as u64, require_both_end as u8,
                              wildcard.map_or(-1, |w| w as i32)) as usize
    }
}
