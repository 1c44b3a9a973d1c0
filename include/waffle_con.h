/*
 * waffle_con MI355X library — C ABI (the drop-in boundary).
 *
 * The reference (PacificBiosciences/waffle_con v0.4.4) is a Rust crate with no
 * FFI; its public API is ConsensusDWFA / DualConsensusDWFA /
 * PriorityConsensusDWFA + CdwfaConfig. A Rust shim keeps that
 * API and calls these entry points; consensus() of each engine maps to one
 * wc_service_* call (many host threads share the device) or to wc_*_batch
 * calls over many problems at once (throughput).
 *
 * Conventions: return 0 = OK, otherwise a WC_E_* code; wc_last_error() holds
 * the message. Caller owns inputs (copied during the call); result sets are
 * owned by the library until wc_results_free. A context is bound to one HIP
 * device and must be used from one host thread at a time.
 */
#ifndef WAFFLE_CON_H
#define WAFFLE_CON_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* error codes; messages match the reference's bail!/panic sites */
enum {
  WC_OK = 0,
  WC_E_FINALIZE_UNINIT = 1, /* consensus.rs:473, dual_consensus.rs:1078 */
  WC_E_NO_START = 2,        /* consensus.rs:205, dual_consensus.rs:303 */
  WC_E_COVERAGE_GAP = 3,    /* consensus.rs:305 */
  WC_E_CAPACITY = 4,        /* pqueue_tracker.rs:90 */
  WC_E_LOCKED = 5,          /* dual_consensus.rs:917,919 */
  WC_E_DUAL_TWICE = 6,      /* dual_consensus.rs:959 */
  WC_E_SAME_SYMBOL = 7,     /* dual_consensus.rs:964 */
  WC_E_ROOT_INACTIVE = 8,   /* consensus.rs:396, dual_consensus.rs:843 */
  WC_E_BAD_INPUT = 9,       /* priority_consensus.rs:144,148; empty inputs */
  WC_E_INVARIANT = 10,      /* reference assert!/panic sites */
  WC_E_LIMIT = 11,          /* a device capacity limit was exceeded after retries. Hard limits
                             * (the reference has none): at most 8 distinct symbols at one read's
                             * wavefront tips, 14 distinct voted symbols per node side and 64
                             * children per node (DNA plus a wildcard and N needs 6). Wavefront,
                             * node-pool, consensus and result capacities grow by retry instead. */
  WC_E_HIP = 12,            /* HIP runtime failure (no device, launch failure) */
};

/* cdwfa_config.rs:38-103 (CdwfaConfig); wc_config_default gives :71-103 */
typedef struct wc_config {
  int32_t consensus_cost; /* 0 = L1Distance, 1 = L2Distance */
  int32_t wildcard;       /* -1 = None, else the wildcard byte */
  uint64_t max_queue_size;
  uint64_t max_capacity_per_size;
  uint64_t max_return_size;
  uint64_t max_nodes_wo_constraint;
  uint64_t min_count;
  double min_af;
  uint64_t dual_max_ed_delta;
  uint64_t offset_window;
  uint64_t offset_compare_length;
  uint8_t weighted_by_ed;
  uint8_t allow_early_termination;
  uint8_t auto_shift_offsets;
  uint8_t _pad[5];
} wc_config;

void wc_config_default(wc_config* cfg);

typedef struct wc_ctx wc_ctx;
typedef struct wc_results wc_results;

int wc_ctx_create(int device, wc_ctx** out);
void wc_ctx_destroy(wc_ctx* ctx);
const char* wc_last_error(const wc_ctx* ctx);
/* Which engine builds this context has launched (no reference counterpart:
 * the reference has one CPU implementation). Bit k = build k, named by
 * wc_engine_name(k) ("lds.single", "wave.dual", ...; NULL past the last);
 * reset != 0 clears the mask after reading it. wc_service_engines_used is the
 * same for a service's own context. */
uint32_t wc_engines_used(wc_ctx* ctx, int reset);
const char* wc_engine_name(uint32_t bit);
/* Bytes the last batch upload of this context sent 2-bit packed (SURVEY §8(f)
 * f3; 0 = it took the byte path: small, WC_PACK=0, or a byte outside the
 * raw-code / ACGT alphabets). */
uint64_t wc_last_upload_packed(const wc_ctx* ctx);

/* One consensus problem (a locus): its reads and optional activation offsets
 * (add_sequence_offset, consensus.rs:120; NULL or -1 entries = None). */
typedef struct wc_problem {
  uint32_t n_reads;
  const uint8_t* const* reads;
  const uint64_t* lens;
  const int64_t* offsets;
} wc_problem;

/* One priority problem: n_chains read chains of `levels` sequences each,
 * row-major (reads[i*levels + l]); offsets likewise (NULL = all None);
 * seed_groups[i] (-1 = None, NULL = all None). priority_consensus.rs:141-167. */
typedef struct wc_chain_problem {
  uint32_t n_chains;
  uint32_t levels;
  const uint8_t* const* reads;
  const uint64_t* lens;
  const int64_t* offsets;
  const int64_t* seed_groups;
} wc_chain_problem;

/* Batched engines: every problem runs the reference search bit-exactly; the
 * whole batch is resident in HBM and runs as one device-resident launch
 * (one workgroup per problem). Per-problem failures are reported through
 * wc_results_status, not the return value. Replaces:
 *   ConsensusDWFA::consensus          consensus.rs:139
 *   DualConsensusDWFA::consensus      dual_consensus.rs:240
 *   PriorityConsensusDWFA::consensus  priority_consensus.rs:172 */
int wc_consensus_batch(wc_ctx* ctx, const wc_config* cfg, uint32_t n, const wc_problem* problems,
                       wc_results** out);
int wc_dual_consensus_batch(wc_ctx* ctx, const wc_config* cfg, uint32_t n, const wc_problem* problems,
                            wc_results** out);
int wc_priority_consensus_batch(wc_ctx* ctx, const wc_config* cfg, uint32_t n, const wc_chain_problem* problems,
                                wc_results** out);

/* Resident batches: upload the reads of many problems to HBM once, then run
 * any engine over them repeatedly (the throughput path; bench.py times
 * wc_batch_consensus with the reads already resident). */
typedef struct wc_batch wc_batch;
int wc_batch_create(wc_ctx* ctx, uint32_t n, const wc_problem* problems, wc_batch** out);
/* Re-uploads a new set of problems into an existing batch, reusing its device
 * buffers when they are large enough (no allocation, so no device-wide
 * synchronisation): the streaming / double-buffered input path. */
int wc_batch_refill(wc_ctx* ctx, wc_batch* b, uint32_t n, const wc_problem* problems);
void wc_batch_free(wc_batch* b);
uint64_t wc_batch_bytes(const wc_batch* b);
int wc_batch_consensus(wc_ctx* ctx, wc_batch* b, const wc_config* cfg, wc_results** out);
int wc_batch_dual_consensus(wc_ctx* ctx, wc_batch* b, const wc_config* cfg, wc_results** out);

/* Submission service: the reference's per-locus API from any number of host
 * threads. ConsensusDWFA::consensus (consensus.rs:139) and
 * DualConsensusDWFA::consensus (dual_consensus.rs:240) are `&self`, re-entrant
 * and one instance per thread; a caller binds them here instead of one
 * wc_*_batch call per locus. Concurrent calls share persistent engine launches
 * on the device (one workgroup per in-flight locus; service.cpp), each call
 * blocks until its own result is ready and returns a one-problem result set
 * (free with wc_results_free), exactly what wc_consensus_batch /
 * wc_dual_consensus_batch with that one problem return. Thread-safe; one
 * service per device. arena_bytes: pinned host memory for the reads of the
 * calls in flight (0 = 256 MiB; a locus larger than a quarter of it takes the
 * batch path). wc_service_priority_consensus serves
 * PriorityConsensusDWFA::consensus (priority_consensus.rs:172-341) the same
 * way: the calling thread unwinds the reference's LIFO work stack and every
 * DualConsensusDWFA sub-problem runs in the shared launches; the result is
 * what wc_priority_consensus_batch with that one problem returns. Calls made
 * while wc_service_destroy runs fail with WC_E_HIP; calls already inside
 * complete first. */
typedef struct wc_service wc_service;
typedef struct wc_service_stats {
  uint64_t calls;       /* consensus calls */
  uint64_t served;      /* answered by the persistent launches */
  uint64_t fallback;    /* answered by the batch path (offsets, > 256 reads, capacity retries) */
  uint64_t lane_starts; /* persistent launches started */
  uint64_t retried;     /* of the fallbacks: problems that outgrew the launch's capacities */
  uint64_t lane_failures; /* launches that could not start (their requests took the batch path) */
} wc_service_stats;
int wc_service_create(int device, uint64_t arena_bytes, wc_service** out);
void wc_service_destroy(wc_service* s);
int wc_service_consensus(wc_service* s, const wc_config* cfg, const wc_problem* problem, wc_results** out);
int wc_service_dual_consensus(wc_service* s, const wc_config* cfg, const wc_problem* problem, wc_results** out);
int wc_service_priority_consensus(wc_service* s, const wc_config* cfg, const wc_chain_problem* problem,
                                  wc_results** out);
uint32_t wc_service_engines_used(wc_service* svc, int reset);
int wc_service_get_stats(wc_service* s, wc_service_stats* out);
const char* wc_service_last_error(wc_service* s);

void wc_results_free(wc_results* r);
uint32_t wc_results_problems(const wc_results* r);
int wc_results_status(const wc_results* r, uint32_t p);
const char* wc_results_error(const wc_results* r, uint32_t p);
uint32_t wc_results_count(const wc_results* r, uint32_t p);

/* Consensus (consensus.rs:42-74): sequence bytes + per-read scores. Pointers
 * stay valid until wc_results_free. */
int wc_results_single(const wc_results* r, uint32_t p, uint32_t k, const uint8_t** seq, uint64_t* seq_len,
                      const uint64_t** scores, uint64_t* n_scores);

/* Every Consensus of a single-consensus result set in one call (a binding
 * helper for many loci; no reference counterpart: it returns what
 * wc_results_status/count/single return, in bulk). wc_results_single_sizes
 * gives the totals over all problems; wc_results_single_pack then fills
 * status[problems], count[problems], seq[seq_bytes] (all sequences back to
 * back), seq_off[n_results + 1], scores[n_scores], score_off[n_results + 1],
 * results in problem order. */
int wc_results_single_sizes(const wc_results* r, uint64_t* n_results, uint64_t* seq_bytes, uint64_t* n_scores);
/* The same results without copies: pointers into arrays the result set owns
 * (valid until wc_results_free): status[problems], count[problems], the
 * sequence and score arenas, and per result (problem order) four u64: sequence
 * start and length in `seq`, scores start and length in `scores`. */
int wc_results_single_view(wc_results* r, const int32_t** status, const uint32_t** count, const uint8_t** seq,
                           const uint64_t** scores, const uint64_t** index);
int wc_results_single_pack(const wc_results* r, int32_t* status, uint32_t* count, uint8_t* seq, uint64_t* seq_off,
                           uint64_t* scores, uint64_t* score_off);

/* DualConsensus (dual_consensus.rs:52-177). scores1/scores2 use -1 for None. */
typedef struct wc_dual_view {
  const uint8_t* seq1;
  uint64_t len1;
  const uint64_t* scores_c1; /* Consensus::scores of consensus1 */
  uint64_t n_scores_c1;
  uint8_t has_c2;
  const uint8_t* seq2;
  uint64_t len2;
  const uint64_t* scores_c2;
  uint64_t n_scores_c2;
  const uint8_t* is_consensus1; /* n_reads */
  const int64_t* scores1;       /* n_reads, -1 = None */
  const int64_t* scores2;
  uint64_t n_reads;
} wc_dual_view;
int wc_results_dual(const wc_results* r, uint32_t p, uint32_t k, wc_dual_view* out);

/* PriorityConsensus (priority_consensus.rs:64-88): for chain k of problem p,
 * wc_results_count gives the number of chains; each chain has `levels`
 * consensuses (wc_results_chain_len). sequence_indices has n_chains entries. */
uint32_t wc_results_chain_len(const wc_results* r, uint32_t p, uint32_t k);
int wc_results_chain(const wc_results* r, uint32_t p, uint32_t k, uint32_t level, const uint8_t** seq,
                     uint64_t* seq_len, const uint64_t** scores, uint64_t* n_scores);
int wc_results_sequence_indices(const wc_results* r, uint32_t p, const uint64_t** idx, uint64_t* n);

/* Work counters and timings of the run that produced `r`. */
typedef struct wc_stats {
  uint64_t updates;      /* DWFALite::update-equivalent calls */
  uint64_t w_out;        /* sum of post-update wavefront lengths */
  uint64_t compares;     /* byte compares the reference extend would make */
  uint64_t ed_increases; /* increase_edit_distance calls */
  uint64_t finalizes;    /* DWFALite::finalize calls */
  uint64_t pops;
  uint64_t nodes_explored;
  uint64_t nodes_ignored;
  uint64_t peak_queue_size; /* max over problems */
  uint64_t row_bytes;       /* wavefront-row bytes read + written by updates (finalizes: read) that grow an
                             * edit distance: the rows' share of the roofline model */
  uint64_t launches;        /* engine kernel launches (incl. capacity retries) */
  double kernel_ms;         /* device time of the engine launches (HIP events) */
  double wall_ms;           /* host wall time of the whole call */
  double start_ms;          /* per problem (wc_results_problem_stats): when its first engine work was
                             * published to the device, from the start of the call (PriorityConsensusDWFA
                             * batches; 0 elsewhere): wall_ms - start_ms is its latency on the device */
} wc_stats;
int wc_results_stats(const wc_results* r, wc_stats* out);
/* per-problem counters (same fields; kernel_ms and launches zero; wall_ms =
 * time from the start of the call until this problem's result was final) */
int wc_results_problem_stats(const wc_results* r, uint32_t p, wc_stats* out);

/* Standalone DWFALite (dynamic_wfa.rs:48-265) on the device: one job = one
 * read-DWFA state advanced by `op` against (baseline, other). Batched: one
 * wave per job. State in/out: e, wavefront[0..wf_len) (capacity wf_cap). */
typedef struct wc_dwfa_job {
  const uint8_t* baseline;
  uint64_t baseline_len;
  const uint8_t* other;
  uint64_t other_len;
  uint64_t offset;
  int32_t wildcard;       /* -1 = None */
  uint8_t early;          /* allow_early_termination */
  uint8_t op;             /* 0 = update, 1 = finalize, 2 = candidates (read-only) */
  uint8_t _pad[2];
  uint64_t e;             /* in/out */
  uint64_t* wavefront;    /* in/out, host memory */
  uint64_t wf_len;        /* in/out */
  uint64_t wf_cap;
  /* op 2 output: symbols in FxHashMap iteration order with counts */
  uint8_t cand_syms[16];
  uint64_t cand_counts[16];
  uint32_t n_cand;
  int32_t status;
  /* op 2 output: the same n_cand symbols in insertion order (first tip in
   * ascending diagonal index: the order of the reference's entry().or_insert()
   * calls, dynamic_wfa.rs:244-250). A hashbrown map's layout depends on it when
   * keys collide (C and G share bucket 3 of 4), so a caller
   * that rebuilds the map inserts in this order. */
  uint8_t cand_first[16];
} wc_dwfa_job;
int wc_dwfa_batch(wc_ctx* ctx, uint32_t n, wc_dwfa_job* jobs);

/* example_gen.rs:11-64 generate_test with the reference RNG (StdRng::seed_from_u64);
 * the reference hardcodes seed 0. Writes consensus (seq_len bytes) and samples
 * into library-owned storage returned through *handle (free with wc_gen_free). */
typedef struct wc_gen wc_gen;
int wc_generate_test(uint8_t alphabet, uint64_t seq_len, uint64_t num_samples, double error_rate, uint64_t seed,
                     wc_gen** handle);
const uint8_t* wc_gen_consensus(const wc_gen* g, uint64_t* len);
const uint8_t* wc_gen_sample(const wc_gen* g, uint64_t i, uint64_t* len);
void wc_gen_free(wc_gen* g);

/* sequence_alignment.rs:18,36 — pairwise WFA edit distance (host reference API). */
uint64_t wc_wfa_ed_config(const uint8_t* v1, uint64_t l1, const uint8_t* v2, uint64_t l2, uint8_t require_both_end,
                          int32_t wildcard);

/* sequence_alignment.rs:18-87 — wfa_ed_config over a batch of pairs on the
 * device (one wave64 per pair): out_ed[i] = wfa_ed_config(v1[i], v2[i],
 * require_both_end, wildcard); wildcard < 0 = None; wfa_ed is
 * (require_both_end = 1, wildcard = '*'). Lengths must be < 2^31. Inputs are
 * host buffers, copied during the call. Returns WC_OK or an error code. */
int wc_wfa_ed_batch(wc_ctx* ctx, uint32_t n, const uint8_t* const* v1, const uint64_t* l1, const uint8_t* const* v2,
                    const uint64_t* l2, uint8_t require_both_end, int32_t wildcard, uint64_t* out_ed);

#ifdef __cplusplus
}
#endif
#endif
