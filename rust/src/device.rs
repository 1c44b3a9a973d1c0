//! Device access for the public API: the per-process submission service of the
//! device (`wc_service_*`), batched calls over many loci, and the decoding of
//! result sets into the reference's result types.
use std::ffi::CStr;
use std::os::raw::c_int;
use std::sync::OnceLock;

use crate::cdwfa_config::{CdwfaConfig, ConsensusCost};
use crate::consensus::Consensus;
use crate::dual_consensus::DualConsensus;
use crate::ffi;
use crate::priority_consensus::PriorityConsensus;

/// An error of the device library: the reference's message for the reference's
/// error cases (include/waffle_con.h WC_E_*), else the library's.
#[derive(Debug, Clone)]
pub struct WcError {
    pub code: i32,
    pub message: String,
}

impl std::fmt::Display for WcError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        f.write_str(&self.message)
    }
}

impl std::error::Error for WcError {}

pub(crate) fn err(code: c_int, message: String) -> Box<dyn std::error::Error> {
    Box::new(WcError { code, message })
}

pub(crate) unsafe fn cstr(p: *const std::os::raw::c_char) -> String {
    if p.is_null() {
        String::new()
    } else {
        CStr::from_ptr(p).to_string_lossy().into_owned()
    }
}

/// The device every call of this process uses: WAFFLE_CON_DEVICE, default 0.
pub fn device_index() -> c_int {
    std::env::var("WAFFLE_CON_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(0)
}

struct Service(*mut ffi::wc_service);
// the service is thread-safe (include/waffle_con.h)
unsafe impl Send for Service {}
unsafe impl Sync for Service {}

static SERVICE: OnceLock<Result<Service, WcError>> = OnceLock::new();

/// The process-wide submission service of the device (created on first use).
fn service() -> Result<*mut ffi::wc_service, Box<dyn std::error::Error>> {
    let s = SERVICE.get_or_init(|| unsafe {
        let mut h = std::ptr::null_mut();
        let rc = ffi::wc_service_create(device_index(), 0, &mut h);
        if rc != ffi::WC_OK {
            Err(WcError { code: rc, message: format!("no usable MI355X (HIP device {})", device_index()) })
        } else {
            Ok(Service(h))
        }
    });
    match s {
        Ok(svc) => Ok(svc.0),
        Err(e) => Err(Box::new(e.clone())),
    }
}

/// Frees a result set when dropped.
pub(crate) struct Results(pub *mut ffi::wc_results);

impl Drop for Results {
    fn drop(&mut self) {
        if !self.0.is_null() {
            unsafe { ffi::wc_results_free(self.0) }
        }
    }
}

/// One wc_problem over borrowed reads (kept alive by this struct).
pub(crate) struct Problem {
    ptrs: Vec<*const u8>,
    lens: Vec<u64>,
    offs: Vec<i64>,
}

impl Problem {
    /// One offset per read (the C library reads `n_reads` of each array, so a
    /// short offsets vector would be read past its end: refused here).
    pub fn new(reads: &[&[u8]], offsets: &[Option<usize>]) -> Result<Problem, Box<dyn std::error::Error>> {
        if offsets.len() != reads.len() {
            return Err(err(ffi::WC_E_BAD_INPUT,
                           format!("expected {} offsets (one per read), got {}", reads.len(), offsets.len())));
        }
        Ok(Problem {
            ptrs: reads.iter().map(|s| s.as_ptr()).collect(),
            lens: reads.iter().map(|s| s.len() as u64).collect(),
            offs: offsets.iter().map(|o| o.map_or(-1, |v| v as i64)).collect(),
        })
    }

    pub fn raw(&self) -> ffi::wc_problem {
        ffi::wc_problem {
            n_reads: self.ptrs.len() as u32,
            reads: self.ptrs.as_ptr(),
            lens: self.lens.as_ptr(),
            offsets: if self.offs.iter().any(|&o| o >= 0) { self.offs.as_ptr() } else { std::ptr::null() },
        }
    }
}

/// One wc_chain_problem (PriorityConsensusDWFA): chains of `levels` reads, row-major.
pub(crate) struct ChainProblem {
    levels: u32,
    ptrs: Vec<*const u8>,
    lens: Vec<u64>,
    offs: Vec<i64>,
    groups: Vec<i64>,
}

impl ChainProblem {
    /// Every chain has the first chain's level count, one offset per (chain,
    /// level) and one seed group per chain: the C library reads `n_chains x
    /// levels` entries of each array, so ragged input would be read past its
    /// end. The reference would panic indexing it (priority_consensus.rs:172-341);
    /// here it is an error.
    pub fn new(chains: &[Vec<&[u8]>], offsets: &[Vec<Option<usize>>], groups: &[Option<usize>])
               -> Result<ChainProblem, Box<dyn std::error::Error>> {
        let levels = chains.first().map_or(0, |c| c.len());
        let bad = |m: String| Err(err(ffi::WC_E_BAD_INPUT, m));
        if let Some(i) = chains.iter().position(|c| c.len() != levels) {
            return bad(format!("sequence chain {} has {} levels, expected {}", i, chains[i].len(), levels));
        }
        if offsets.len() != chains.len() {
            return bad(format!("expected {} offset vectors (one per chain), got {}", chains.len(), offsets.len()));
        }
        if let Some(i) = offsets.iter().position(|o| o.len() != levels) {
            return bad(format!("offsets of chain {} have {} entries, expected {}", i, offsets[i].len(), levels));
        }
        if groups.len() != chains.len() {
            return bad(format!("expected {} seed groups (one per chain), got {}", chains.len(), groups.len()));
        }
        Ok(ChainProblem {
            levels: levels as u32,
            ptrs: chains.iter().flat_map(|c| c.iter().map(|s| s.as_ptr())).collect(),
            lens: chains.iter().flat_map(|c| c.iter().map(|s| s.len() as u64)).collect(),
            offs: offsets.iter().flat_map(|c| c.iter().map(|o| o.map_or(-1, |v| v as i64))).collect(),
            groups: groups.iter().map(|g| g.map_or(-1, |v| v as i64)).collect(),
        })
    }

    pub fn raw(&self) -> ffi::wc_chain_problem {
        ffi::wc_chain_problem {
            n_chains: self.groups.len() as u32,
            levels: self.levels,
            reads: self.ptrs.as_ptr(),
            lens: self.lens.as_ptr(),
            offsets: if self.offs.iter().any(|&o| o >= 0) { self.offs.as_ptr() } else { std::ptr::null() },
            seed_groups: if self.groups.iter().any(|&g| g >= 0) { self.groups.as_ptr() } else { std::ptr::null() },
        }
    }
}

fn check_problem(res: &Results, p: u32) -> Result<(), Box<dyn std::error::Error>> {
    unsafe {
        let st = ffi::wc_results_status(res.0, p);
        if st != ffi::WC_OK {
            return Err(err(st, cstr(ffi::wc_results_error(res.0, p))));
        }
    }
    Ok(())
}

unsafe fn slice<'b, T>(p: *const T, n: u64) -> &'b [T] {
    if n == 0 {
        &[]
    } else {
        std::slice::from_raw_parts(p, n as usize)
    }
}

/// consensus.rs:139 results of problem p
pub(crate) fn decode_single(res: &Results, p: u32, cost: ConsensusCost) -> Result<Vec<Consensus>, Box<dyn std::error::Error>> {
    check_problem(res, p)?;
    let mut out = Vec::new();
    unsafe {
        for k in 0..ffi::wc_results_count(res.0, p) {
            let (mut s, mut sl, mut sc, mut scl) = (std::ptr::null(), 0u64, std::ptr::null(), 0u64);
            ffi::wc_results_single(res.0, p, k, &mut s, &mut sl, &mut sc, &mut scl);
            out.push(Consensus::new(slice(s, sl).to_vec(), cost, slice(sc, scl).iter().map(|&v| v as usize).collect()));
        }
    }
    Ok(out)
}

/// dual_consensus.rs:240 results of problem p
pub(crate) fn decode_dual(res: &Results, p: u32, cost: ConsensusCost) -> Result<Vec<DualConsensus>, Box<dyn std::error::Error>> {
    check_problem(res, p)?;
    let mut out = Vec::new();
    unsafe {
        for k in 0..ffi::wc_results_count(res.0, p) {
            let mut v: ffi::wc_dual_view = std::mem::zeroed();
            ffi::wc_results_dual(res.0, p, k, &mut v);
            let c1 = Consensus::new(slice(v.seq1, v.len1).to_vec(), cost,
                                    slice(v.scores_c1, v.n_scores_c1).iter().map(|&x| x as usize).collect());
            let c2 = if v.has_c2 != 0 {
                Some(Consensus::new(slice(v.seq2, v.len2).to_vec(), cost,
                                    slice(v.scores_c2, v.n_scores_c2).iter().map(|&x| x as usize).collect()))
            } else {
                None
            };
            let opt = |x: &i64| if *x < 0 { None } else { Some(*x as usize) };
            let d = DualConsensus::new(c1, c2, slice(v.is_consensus1, v.n_reads).iter().map(|&b| b != 0).collect(),
                                       slice(v.scores1, v.n_reads).iter().map(opt).collect(),
                                       slice(v.scores2, v.n_reads).iter().map(opt).collect())?;
            out.push(d);
        }
    }
    Ok(out)
}

/// priority_consensus.rs:172 result of problem p
pub(crate) fn decode_priority(res: &Results, p: u32, cost: ConsensusCost) -> Result<PriorityConsensus, Box<dyn std::error::Error>> {
    check_problem(res, p)?;
    unsafe {
        let mut chains = Vec::new();
        for k in 0..ffi::wc_results_count(res.0, p) {
            let mut chain = Vec::new();
            for l in 0..ffi::wc_results_chain_len(res.0, p, k) {
                let (mut s, mut sl, mut sc, mut scl) = (std::ptr::null(), 0u64, std::ptr::null(), 0u64);
                ffi::wc_results_chain(res.0, p, k, l, &mut s, &mut sl, &mut sc, &mut scl);
                chain.push(Consensus::new(slice(s, sl).to_vec(), cost, slice(sc, scl).iter().map(|&v| v as usize).collect()));
            }
            chains.push(chain);
        }
        let (mut ip, mut il) = (std::ptr::null(), 0u64);
        ffi::wc_results_sequence_indices(res.0, p, &mut ip, &mut il);
        Ok(PriorityConsensus::new(chains, slice(ip, il).iter().map(|&v| v as usize).collect()))
    }
}

fn svc_err(s: *mut ffi::wc_service, rc: c_int) -> Box<dyn std::error::Error> {
    err(rc, unsafe { cstr(ffi::wc_service_last_error(s)) })
}

/// One ConsensusDWFA::consensus through the service
pub(crate) fn service_single(cfg: &CdwfaConfig, prob: &Problem) -> Result<Vec<Consensus>, Box<dyn std::error::Error>> {
    let s = service()?;
    let (c, p) = (cfg.to_wc(), prob.raw());
    let mut r = std::ptr::null_mut();
    let rc = unsafe { ffi::wc_service_consensus(s, &c, &p, &mut r) };
    if rc != ffi::WC_OK {
        return Err(svc_err(s, rc));
    }
    decode_single(&Results(r), 0, cfg.consensus_cost)
}

/// One DualConsensusDWFA::consensus through the service
pub(crate) fn service_dual(cfg: &CdwfaConfig, prob: &Problem) -> Result<Vec<DualConsensus>, Box<dyn std::error::Error>> {
    let s = service()?;
    let (c, p) = (cfg.to_wc(), prob.raw());
    let mut r = std::ptr::null_mut();
    let rc = unsafe { ffi::wc_service_dual_consensus(s, &c, &p, &mut r) };
    if rc != ffi::WC_OK {
        return Err(svc_err(s, rc));
    }
    decode_dual(&Results(r), 0, cfg.consensus_cost)
}

/// One PriorityConsensusDWFA::consensus through the service
pub(crate) fn service_priority(cfg: &CdwfaConfig, prob: &ChainProblem) -> Result<PriorityConsensus, Box<dyn std::error::Error>> {
    let s = service()?;
    let (c, p) = (cfg.to_wc(), prob.raw());
    let mut r = std::ptr::null_mut();
    let rc = unsafe { ffi::wc_service_priority_consensus(s, &c, &p, &mut r) };
    if rc != ffi::WC_OK {
        return Err(svc_err(s, rc));
    }
    decode_priority(&Results(r), 0, cfg.consensus_cost)
}

/// A context of this thread (batched calls)
struct Ctx(*mut ffi::wc_ctx);

impl Drop for Ctx {
    fn drop(&mut self) {
        unsafe { ffi::wc_ctx_destroy(self.0) }
    }
}

thread_local! {
    static CTX: std::cell::RefCell<Option<Ctx>> = const { std::cell::RefCell::new(None) };
}

pub(crate) fn with_ctx<T>(f: impl FnOnce(*mut ffi::wc_ctx) -> Result<T, Box<dyn std::error::Error>>) -> Result<T, Box<dyn std::error::Error>> {
    CTX.with(|c| {
        let mut c = c.borrow_mut();
        if c.is_none() {
            let mut h = std::ptr::null_mut();
            let rc = unsafe { ffi::wc_ctx_create(device_index(), &mut h) };
            if rc != ffi::WC_OK {
                return Err(err(rc, format!("no usable MI355X (HIP device {})", device_index())));
            }
            *c = Some(Ctx(h));
        }
        f(c.as_ref().unwrap().0)
    })
}

/// ConsensusDWFA::consensus for many loci in one launch (each locus: its reads
/// and offsets). Per-locus errors are returned per locus.
pub fn consensus_batch(cfg: &CdwfaConfig, loci: &[(Vec<&[u8]>, Vec<Option<usize>>)])
                       -> Result<Vec<Result<Vec<Consensus>, Box<dyn std::error::Error>>>, Box<dyn std::error::Error>> {
    let probs: Vec<Problem> = loci.iter().map(|(r, o)| Problem::new(r, o)).collect::<Result<_, _>>()?;
    let raw: Vec<ffi::wc_problem> = probs.iter().map(|p| p.raw()).collect();
    let c = cfg.to_wc();
    with_ctx(|ctx| {
        let mut r = std::ptr::null_mut();
        let rc = unsafe { ffi::wc_consensus_batch(ctx, &c, raw.len() as u32, raw.as_ptr(), &mut r) };
        if rc != ffi::WC_OK {
            return Err(err(rc, unsafe { cstr(ffi::wc_last_error(ctx)) }));
        }
        let res = Results(r);
        Ok((0..raw.len() as u32).map(|p| decode_single(&res, p, cfg.consensus_cost)).collect())
    })
}

/// DualConsensusDWFA::consensus for many loci in one launch.
pub fn dual_consensus_batch(cfg: &CdwfaConfig, loci: &[(Vec<&[u8]>, Vec<Option<usize>>)])
                            -> Result<Vec<Result<Vec<DualConsensus>, Box<dyn std::error::Error>>>, Box<dyn std::error::Error>> {
    let probs: Vec<Problem> = loci.iter().map(|(r, o)| Problem::new(r, o)).collect::<Result<_, _>>()?;
    let raw: Vec<ffi::wc_problem> = probs.iter().map(|p| p.raw()).collect();
    let c = cfg.to_wc();
    with_ctx(|ctx| {
        let mut r = std::ptr::null_mut();
        let rc = unsafe { ffi::wc_dual_consensus_batch(ctx, &c, raw.len() as u32, raw.as_ptr(), &mut r) };
        if rc != ffi::WC_OK {
            return Err(err(rc, unsafe { cstr(ffi::wc_last_error(ctx)) }));
        }
        let res = Results(r);
        Ok((0..raw.len() as u32).map(|p| decode_dual(&res, p, cfg.consensus_cost)).collect())
    })
}

/// PriorityConsensusDWFA::consensus for many loci in one streamed launch
/// (each locus: its chains, per-level offsets and seed groups).
#[allow(clippy::type_complexity)]
pub fn priority_consensus_batch(cfg: &CdwfaConfig, loci: &[(Vec<Vec<&[u8]>>, Vec<Vec<Option<usize>>>, Vec<Option<usize>>)])
                                -> Result<Vec<Result<PriorityConsensus, Box<dyn std::error::Error>>>, Box<dyn std::error::Error>> {
    let probs: Vec<ChainProblem> = loci.iter().map(|(c, o, g)| ChainProblem::new(c, o, g)).collect::<Result<_, _>>()?;
    let raw: Vec<ffi::wc_chain_problem> = probs.iter().map(|p| p.raw()).collect();
    let c = cfg.to_wc();
    with_ctx(|ctx| {
        let mut r = std::ptr::null_mut();
        let rc = unsafe { ffi::wc_priority_consensus_batch(ctx, &c, raw.len() as u32, raw.as_ptr(), &mut r) };
        if rc != ffi::WC_OK {
            return Err(err(rc, unsafe { cstr(ffi::wc_last_error(ctx)) }));
        }
        let res = Results(r);
        Ok((0..raw.len() as u32).map(|p| decode_priority(&res, p, cfg.consensus_cost)).collect())
    })
}

/// sequence_alignment.rs:18-87 over many pairs on the device
pub fn wfa_ed_batch(pairs: &[(&[u8], &[u8])], require_both_end: bool, wildcard: Option<u8>)
                    -> Result<Vec<usize>, Box<dyn std::error::Error>> {
    let v1: Vec<*const u8> = pairs.iter().map(|p| p.0.as_ptr()).collect();
    let l1: Vec<u64> = pairs.iter().map(|p| p.0.len() as u64).collect();
    let v2: Vec<*const u8> = pairs.iter().map(|p| p.1.as_ptr()).collect();
    let l2: Vec<u64> = pairs.iter().map(|p| p.1.len() as u64).collect();
    let mut out = vec![0u64; pairs.len()];
    with_ctx(|ctx| {
        let rc = unsafe {
            ffi::wc_wfa_ed_batch(ctx, pairs.len() as u32, v1.as_ptr(), l1.as_ptr(), v2.as_ptr(), l2.as_ptr(),
                                 require_both_end as u8, wildcard.map_or(-1, |w| w as i32), out.as_mut_ptr())
        };
        if rc != ffi::WC_OK {
            return Err(err(rc, unsafe { cstr(ffi::wc_last_error(ctx)) }));
        }
        Ok(out.iter().map(|&v| v as usize).collect())
    })
}
