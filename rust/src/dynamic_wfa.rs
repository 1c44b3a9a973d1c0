//! DWFALite (dynamic_wfa.rs:12-265): one read's dynamic-WFA state, the same
//! fields, constructors, accessors and errors. `update`, `finalize` and
//! `get_extension_candidates` run on the MI355X (`wc_dwfa_batch`: one wave per
//! job, lanes over the wavefront's diagonals, the same kernels the consensus
//! engines use); the state lives on the host between calls, so `clone()` and
//! the derived `Eq`/`Hash` are plain copies and comparisons, as in the
//! reference.
use rustc_hash::FxHashMap as HashMap;

use crate::device;
use crate::ffi;

/// dynamic_wfa.rs:12-32
#[derive(Clone, Debug, Eq, Hash, PartialEq)]
pub struct DWFALite {
    edit_distance: usize,
    wavefront: Vec<usize>,
    is_finalized: bool,
    wildcard: Option<u8>,
    allow_early_termination: bool,
    offset: usize,
}

/// dynamic_wfa.rs:34-45
impl Default for DWFALite {
    fn default() -> Self {
        DWFALite { edit_distance: 0, wavefront: vec![0], is_finalized: false, wildcard: None,
                   allow_early_termination: false, offset: 0 }
    }
}

/// wc_dwfa_job::op
const OP_UPDATE: u8 = 0;
const OP_FINALIZE: u8 = 1;
const OP_CANDIDATES: u8 = 2;

impl DWFALite {
    /// dynamic_wfa.rs:52-58
    pub fn new(wildcard: Option<u8>, allow_early_termination: bool) -> DWFALite {
        DWFALite { wildcard, allow_early_termination, ..Default::default() }
    }

    /// dynamic_wfa.rs:64-66
    pub fn set_offset(&mut self, offset: usize) {
        self.offset = offset;
    }

    /// One device job over (baseline, other) from this state. Returns the job
    /// (edit distance, wavefront length, candidates) and the wavefront buffer.
    fn run(&self, baseline_seq: &[u8], other_seq: &[u8], op: u8)
           -> Result<(ffi::wc_dwfa_job, Vec<u64>), Box<dyn std::error::Error>> {
        // the wavefront grows by 2 per edit: 2 * (|baseline| + |other|) + 3 bounds it
        let cap = 256usize.max(2 * (baseline_seq.len() + other_seq.len()) + 3).max(self.wavefront.len());
        let mut wf: Vec<u64> = self.wavefront.iter().map(|&d| d as u64).collect();
        wf.resize(cap, 0);
        let mut job = ffi::wc_dwfa_job {
            baseline: baseline_seq.as_ptr(),
            baseline_len: baseline_seq.len() as u64,
            other: other_seq.as_ptr(),
            other_len: other_seq.len() as u64,
            offset: self.offset as u64,
            wildcard: self.wildcard.map_or(-1, |w| w as i32),
            early: self.allow_early_termination as u8,
            op,
            _pad: [0; 2],
            e: self.edit_distance as u64,
            wavefront: wf.as_mut_ptr(),
            wf_len: self.wavefront.len() as u64,
            wf_cap: cap as u64,
            cand_syms: [0; 16],
            cand_counts: [0; 16],
            n_cand: 0,
            status: 0,
            cand_first: [0; 16],
        };
        device::with_ctx(|ctx| {
            let rc = unsafe { ffi::wc_dwfa_batch(ctx, 1, &mut job) };
            if rc != ffi::WC_OK {
                return Err(device::err(rc, unsafe { device::cstr(ffi::wc_last_error(ctx)) }));
            }
            if job.status != 0 {
                return Err(device::err(job.status, format!("DWFA device job failed (status {})", job.status)));
            }
            Ok(())
        })?;
        Ok((job, wf))
    }

    fn take(&mut self, job: &ffi::wc_dwfa_job, wf: &[u64]) {
        self.edit_distance = job.e as usize;
        self.wavefront = wf[..job.wf_len as usize].iter().map(|&d| d as usize).collect();
    }

    /// dynamic_wfa.rs:75-99: appends what `other_seq` gained since the last
    /// call; returns the edit distance
    pub fn update(&mut self, baseline_seq: &[u8], other_seq: &[u8]) -> Result<usize, Box<dyn std::error::Error>> {
        if self.is_finalized {
            return Err("Cannot push more bases after finalizing a DWFA".into());
        }
        let (job, wf) = self.run(baseline_seq, other_seq, OP_UPDATE)?;
        self.take(&job, &wf);
        Ok(self.edit_distance)
    }

    /// dynamic_wfa.rs:201-210 (as in the reference, it does not mark the DWFA
    /// finalized)
    pub fn finalize(&mut self, baseline_seq: &[u8], other_seq: &[u8]) -> Result<(), Box<dyn std::error::Error>> {
        if self.is_finalized {
            return Err("Cannot finalize a DWFA twice.".into());
        }
        let (job, wf) = self.run(baseline_seq, other_seq, OP_FINALIZE)?;
        self.take(&job, &wf);
        Ok(())
    }

    /// dynamic_wfa.rs:213-220
    pub fn maximum_baseline_distance(&self) -> usize {
        self.wavefront.iter().enumerate().map(|(i, &d)| d + self.edit_distance - i).max().unwrap()
    }

    /// dynamic_wfa.rs:224-227
    pub fn maximum_other_distance(&self) -> usize {
        self.offset + *self.wavefront.iter().max().unwrap()
    }

    /// dynamic_wfa.rs:232-234 (`==`, as in the reference)
    pub fn reached_baseline_end(&self, baseline_seq: &[u8]) -> bool {
        self.maximum_baseline_distance() == baseline_seq.len()
    }

    /// dynamic_wfa.rs:241-255: the symbols at the wavefront's tips with their
    /// counts. The device returns them in FxHashMap iteration order with their
    /// counts, and also in insertion order (first tip in ascending diagonal
    /// index, `cand_first`). The map is rebuilt by inserting in that order, as
    /// the reference's `entry().or_insert()` calls do: a hashbrown table's
    /// layout, and so its iteration order, depends on the insertion order when
    /// keys share a home bucket (C and G in a 4-bucket table, SURVEY Appendix
    /// B). Infallible in the reference: a device failure here panics with the
    /// library's message.
    pub fn get_extension_candidates(&self, baseline_seq: &[u8], other_seq: &[u8]) -> HashMap<u8, usize> {
        let (job, _) = self.run(baseline_seq, other_seq, OP_CANDIDATES)
            .unwrap_or_else(|e| panic!("get_extension_candidates on the device failed: {}", e));
        let n = job.n_cand as usize;
        let count = |s: u8| -> usize {
            (0..n).find(|&k| job.cand_syms[k] == s).map(|k| job.cand_counts[k] as usize)
                .unwrap_or_else(|| panic!("get_extension_candidates: symbol {} missing from the device's map", s))
        };
        let mut ret: HashMap<u8, usize> = Default::default();
        for k in 0..n {
            let s = job.cand_first[k];
            ret.insert(s, count(s));
        }
        ret
    }

    /// dynamic_wfa.rs:258-260
    pub fn edit_distance(&self) -> usize {
        self.edit_distance
    }

    /// dynamic_wfa.rs:262-264
    pub fn wavefront(&self) -> &[usize] {
        &self.wavefront
    }
}
