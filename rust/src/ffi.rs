//! Raw bindings of the MI355X library's C ABI: a transcription of
//! `include/waffle_con.h` (tests/test_rust_crate.py checks every declaration
//! here against the header: names, argument counts, struct fields in order).
#![allow(non_camel_case_types, dead_code)]

use std::os::raw::{c_char, c_int};

pub const WC_OK: c_int = 0;
pub const WC_E_FINALIZE_UNINIT: c_int = 1;
pub const WC_E_NO_START: c_int = 2;
pub const WC_E_COVERAGE_GAP: c_int = 3;
pub const WC_E_CAPACITY: c_int = 4;
pub const WC_E_LOCKED: c_int = 5;
pub const WC_E_DUAL_TWICE: c_int = 6;
pub const WC_E_SAME_SYMBOL: c_int = 7;
pub const WC_E_ROOT_INACTIVE: c_int = 8;
pub const WC_E_BAD_INPUT: c_int = 9;
pub const WC_E_INVARIANT: c_int = 10;
pub const WC_E_LIMIT: c_int = 11;
pub const WC_E_HIP: c_int = 12;

#[repr(C)]
pub struct wc_ctx {
    _p: [u8; 0],
}
#[repr(C)]
pub struct wc_results {
    _p: [u8; 0],
}
#[repr(C)]
pub struct wc_batch {
    _p: [u8; 0],
}
#[repr(C)]
pub struct wc_service {
    _p: [u8; 0],
}
#[repr(C)]
pub struct wc_gen {
    _p: [u8; 0],
}

/// cdwfa_config.rs:38-103 (CdwfaConfig)
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct wc_config {
    pub consensus_cost: i32,
    pub wildcard: i32,
    pub max_queue_size: u64,
    pub max_capacity_per_size: u64,
    pub max_return_size: u64,
    pub max_nodes_wo_constraint: u64,
    pub min_count: u64,
    pub min_af: f64,
    pub dual_max_ed_delta: u64,
    pub offset_window: u64,
    pub offset_compare_length: u64,
    pub weighted_by_ed: u8,
    pub allow_early_termination: u8,
    pub auto_shift_offsets: u8,
    pub _pad: [u8; 5],
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct wc_problem {
    pub n_reads: u32,
    pub reads: *const *const u8,
    pub lens: *const u64,
    pub offsets: *const i64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct wc_chain_problem {
    pub n_chains: u32,
    pub levels: u32,
    pub reads: *const *const u8,
    pub lens: *const u64,
    pub offsets: *const i64,
    pub seed_groups: *const i64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct wc_service_stats {
    pub calls: u64,
    pub served: u64,
    pub fallback: u64,
    pub lane_starts: u64,
    pub retried: u64,
    pub lane_failures: u64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct wc_dual_view {
    pub seq1: *const u8,
    pub len1: u64,
    pub scores_c1: *const u64,
    pub n_scores_c1: u64,
    pub has_c2: u8,
    pub seq2: *const u8,
    pub len2: u64,
    pub scores_c2: *const u64,
    pub n_scores_c2: u64,
    pub is_consensus1: *const u8,
    pub scores1: *const i64,
    pub scores2: *const i64,
    pub n_reads: u64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct wc_stats {
    pub updates: u64,
    pub w_out: u64,
    pub compares: u64,
    pub ed_increases: u64,
    pub finalizes: u64,
    pub pops: u64,
    pub nodes_explored: u64,
    pub nodes_ignored: u64,
    pub peak_queue_size: u64,
    pub row_bytes: u64,
    pub launches: u64,
    pub kernel_ms: f64,
    pub wall_ms: f64,
    pub start_ms: f64,
}

#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct wc_dwfa_job {
    pub baseline: *const u8,
    pub baseline_len: u64,
    pub other: *const u8,
    pub other_len: u64,
    pub offset: u64,
    pub wildcard: i32,
    pub early: u8,
    pub op: u8,
    pub _pad: [u8; 2],
    pub e: u64,
    pub wavefront: *mut u64,
    pub wf_len: u64,
    pub wf_cap: u64,
    pub cand_syms: [u8; 16],
    pub cand_counts: [u64; 16],
    pub n_cand: u32,
    pub status: i32,
    pub cand_first: [u8; 16],
}

extern "C" {
    pub fn wc_config_default(cfg: *mut wc_config);
    pub fn wc_ctx_create(device: c_int, out: *mut *mut wc_ctx) -> c_int;
    pub fn wc_ctx_destroy(ctx: *mut wc_ctx);
    pub fn wc_last_error(ctx: *const wc_ctx) -> *const c_char;
    pub fn wc_engines_used(ctx: *mut wc_ctx, reset: c_int) -> u32;
    pub fn wc_engine_name(bit: u32) -> *const c_char;
    pub fn wc_last_upload_packed(ctx: *const wc_ctx) -> u64;

    pub fn wc_consensus_batch(ctx: *mut wc_ctx, cfg: *const wc_config, n: u32, problems: *const wc_problem,
                              out: *mut *mut wc_results) -> c_int;
    pub fn wc_dual_consensus_batch(ctx: *mut wc_ctx, cfg: *const wc_config, n: u32, problems: *const wc_problem,
                                   out: *mut *mut wc_results) -> c_int;
    pub fn wc_priority_consensus_batch(ctx: *mut wc_ctx, cfg: *const wc_config, n: u32,
                                       problems: *const wc_chain_problem, out: *mut *mut wc_results) -> c_int;

    pub fn wc_batch_create(ctx: *mut wc_ctx, n: u32, problems: *const wc_problem, out: *mut *mut wc_batch) -> c_int;
    pub fn wc_batch_refill(ctx: *mut wc_ctx, b: *mut wc_batch, n: u32, problems: *const wc_problem) -> c_int;
    pub fn wc_batch_free(b: *mut wc_batch);
    pub fn wc_batch_bytes(b: *const wc_batch) -> u64;
    pub fn wc_batch_consensus(ctx: *mut wc_ctx, b: *mut wc_batch, cfg: *const wc_config,
                              out: *mut *mut wc_results) -> c_int;
    pub fn wc_batch_dual_consensus(ctx: *mut wc_ctx, b: *mut wc_batch, cfg: *const wc_config,
                                   out: *mut *mut wc_results) -> c_int;

    pub fn wc_service_create(device: c_int, arena_bytes: u64, out: *mut *mut wc_service) -> c_int;
    pub fn wc_service_destroy(s: *mut wc_service);
    pub fn wc_service_consensus(s: *mut wc_service, cfg: *const wc_config, problem: *const wc_problem,
                                out: *mut *mut wc_results) -> c_int;
    pub fn wc_service_dual_consensus(s: *mut wc_service, cfg: *const wc_config, problem: *const wc_problem,
                                     out: *mut *mut wc_results) -> c_int;
    pub fn wc_service_priority_consensus(s: *mut wc_service, cfg: *const wc_config,
                                         problem: *const wc_chain_problem, out: *mut *mut wc_results) -> c_int;
    pub fn wc_service_get_stats(s: *mut wc_service, out: *mut wc_service_stats) -> c_int;
    pub fn wc_service_last_error(s: *mut wc_service) -> *const c_char;
    pub fn wc_service_engines_used(s: *mut wc_service, reset: c_int) -> u32;

    pub fn wc_results_free(r: *mut wc_results);
    pub fn wc_results_problems(r: *const wc_results) -> u32;
    pub fn wc_results_status(r: *const wc_results, p: u32) -> c_int;
    pub fn wc_results_error(r: *const wc_results, p: u32) -> *const c_char;
    pub fn wc_results_count(r: *const wc_results, p: u32) -> u32;
    pub fn wc_results_single(r: *const wc_results, p: u32, k: u32, seq: *mut *const u8, seq_len: *mut u64,
                             scores: *mut *const u64, n_scores: *mut u64) -> c_int;
    pub fn wc_results_single_sizes(r: *const wc_results, n_results: *mut u64, seq_bytes: *mut u64,
                                   n_scores: *mut u64) -> c_int;
    pub fn wc_results_single_view(r: *mut wc_results, status: *mut *const i32, count: *mut *const u32,
                                  seq: *mut *const u8, scores: *mut *const u64, index: *mut *const u64) -> c_int;
    pub fn wc_results_single_pack(r: *const wc_results, status: *mut i32, count: *mut u32, seq: *mut u8,
                                  seq_off: *mut u64, scores: *mut u64, score_off: *mut u64) -> c_int;
    pub fn wc_results_dual(r: *const wc_results, p: u32, k: u32, out: *mut wc_dual_view) -> c_int;
    pub fn wc_results_chain_len(r: *const wc_results, p: u32, k: u32) -> u32;
    pub fn wc_results_chain(r: *const wc_results, p: u32, k: u32, level: u32, seq: *mut *const u8,
                            seq_len: *mut u64, scores: *mut *const u64, n_scores: *mut u64) -> c_int;
    pub fn wc_results_sequence_indices(r: *const wc_results, p: u32, idx: *mut *const u64, n: *mut u64) -> c_int;
    pub fn wc_results_stats(r: *const wc_results, out: *mut wc_stats) -> c_int;
    pub fn wc_results_problem_stats(r: *const wc_results, p: u32, out: *mut wc_stats) -> c_int;

    pub fn wc_dwfa_batch(ctx: *mut wc_ctx, n: u32, jobs: *mut wc_dwfa_job) -> c_int;

    pub fn wc_generate_test(alphabet: u8, seq_len: u64, num_samples: u64, error_rate: f64, seed: u64,
                            handle: *mut *mut wc_gen) -> c_int;
    pub fn wc_gen_consensus(g: *const wc_gen, len: *mut u64) -> *const u8;
    pub fn wc_gen_sample(g: *const wc_gen, i: u64, len: *mut u64) -> *const u8;
    pub fn wc_gen_free(g: *mut wc_gen);

    pub fn wc_wfa_ed_config(v1: *const u8, l1: u64, v2: *const u8, l2: u64, require_both_end: u8,
                            wildcard: i32) -> u64;
    pub fn wc_wfa_ed_batch(ctx: *mut wc_ctx, n: u32, v1: *const *const u8, l1: *const u64, v2: *const *const u8,
                           l2: *const u64, require_both_end: u8, wildcard: i32, out_ed: *mut u64) -> c_int;
}
