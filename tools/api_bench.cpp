// BENCH INFRASTRUCTURE (tools/Makefile -> tools/libapibench.so; bench.py
// --workload cfg2-api). The reference-API caller of SURVEY §8(b): T host
// threads, each calling ConsensusDWFA::consensus / DualConsensusDWFA::consensus
// (consensus.rs:139, dual_consensus.rs:240) on its own loci, one locus per
// call, as a Rust caller (StarPhase) binding the C ABI would. No GIL: this is
// native threads calling the product library.
//   mode 0: wc_service_consensus / wc_service_dual_consensus (one service)
//   mode 1: one wc_consensus_batch / wc_dual_consensus_batch call per locus on
//           a per-thread context (a small launch per call)
// api_bench_priority_run: the same for PriorityConsensusDWFA::consensus
// (priority_consensus.rs:172), wc_service_priority_consensus (mode 0) or one
// wc_priority_consensus_batch call per locus (mode 1).
// The product library is the one the caller already loaded (dlopen NOLOAD of
// its path), so the harness never brings in a second copy.
#include <dlfcn.h>

#include <cstdio>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

#include "../include/waffle_con.h"

namespace {
template <class F>
bool sym(void* h, const char* name, F& f) {
  f = reinterpret_cast<F>(dlsym(h, name));
  return f != nullptr;
}
}  // namespace

// Runs n loci on `threads` threads; results[i] receives locus i's result set
// (caller frees with wc_results_free), lat_ms[i] its call latency. Returns 0,
// or the first failing call's return code (-1: library symbols not found).
extern "C" int api_bench_run(const char* libpath, int device, int mode, uint32_t threads, uint32_t sides, uint32_t n,
                             const wc_problem* loci, const wc_config* cfg, wc_results** results, double* lat_ms,
                             double* wall_s, wc_service_stats* svc_stats) {
  void* h = dlopen(libpath, RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen(libpath, RTLD_NOW);
  if (!h) return -1;
  decltype(&wc_service_create) svc_create;
  decltype(&wc_service_destroy) svc_destroy;
  decltype(&wc_service_consensus) svc_single;
  decltype(&wc_service_dual_consensus) svc_dual;
  decltype(&wc_service_get_stats) svc_stats_fn;
  decltype(&wc_ctx_create) ctx_create;
  decltype(&wc_ctx_destroy) ctx_destroy;
  decltype(&wc_consensus_batch) batch_single;
  decltype(&wc_dual_consensus_batch) batch_dual;
  if (!sym(h, "wc_service_create", svc_create) || !sym(h, "wc_service_destroy", svc_destroy) ||
      !sym(h, "wc_service_consensus", svc_single) || !sym(h, "wc_service_dual_consensus", svc_dual) ||
      !sym(h, "wc_service_get_stats", svc_stats_fn) || !sym(h, "wc_ctx_create", ctx_create) ||
      !sym(h, "wc_ctx_destroy", ctx_destroy) || !sym(h, "wc_consensus_batch", batch_single) ||
      !sym(h, "wc_dual_consensus_batch", batch_dual))
    return -1;
  wc_service* svc = nullptr;
  if (mode == 0) {
    const int rc = svc_create(device, 0, &svc);
    if (rc) return rc;
  }
  std::atomic<uint32_t> next{0};
  std::atomic<int> first_rc{0};
  auto worker = [&]() {
    wc_ctx* ctx = nullptr;
    if (mode == 1 && ctx_create(device, &ctx) != 0) {
      first_rc = 12;
      return;
    }
    for (;;) {
      const uint32_t i = next++;
      if (i >= n || first_rc.load()) break;
      const auto t0 = std::chrono::steady_clock::now();
      int rc;
      if (mode == 0) rc = sides == 1 ? svc_single(svc, cfg, &loci[i], &results[i]) : svc_dual(svc, cfg, &loci[i], &results[i]);
      else rc = sides == 1 ? batch_single(ctx, cfg, 1, &loci[i], &results[i]) : batch_dual(ctx, cfg, 1, &loci[i], &results[i]);
      lat_ms[i] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (rc) {
        int z = 0;
        first_rc.compare_exchange_strong(z, rc);
      }
    }
    if (ctx) ctx_destroy(ctx);
  };
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < threads; ++t) th.emplace_back(worker);
  for (auto& x : th) x.join();
  *wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (svc) {
    if (svc_stats) svc_stats_fn(svc, svc_stats);
    svc_destroy(svc);
  }
  return first_rc.load();
}

extern "C" int api_bench_priority_run(const char* libpath, int device, int mode, uint32_t threads, uint32_t n,
                                      const wc_chain_problem* loci, const wc_config* cfg, wc_results** results,
                                      double* lat_ms, double* wall_s, wc_service_stats* svc_stats) {
  void* h = dlopen(libpath, RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen(libpath, RTLD_NOW);
  if (!h) return -1;
  decltype(&wc_service_create) svc_create;
  decltype(&wc_service_destroy) svc_destroy;
  decltype(&wc_service_priority_consensus) svc_prio;
  decltype(&wc_service_get_stats) svc_stats_fn;
  decltype(&wc_ctx_create) ctx_create;
  decltype(&wc_ctx_destroy) ctx_destroy;
  decltype(&wc_priority_consensus_batch) batch_prio;
  decltype(&wc_last_error) last_error;
  decltype(&wc_service_last_error) svc_last_error;
  if (!sym(h, "wc_service_create", svc_create) || !sym(h, "wc_service_destroy", svc_destroy) ||
      !sym(h, "wc_service_priority_consensus", svc_prio) || !sym(h, "wc_service_get_stats", svc_stats_fn) ||
      !sym(h, "wc_ctx_create", ctx_create) || !sym(h, "wc_ctx_destroy", ctx_destroy) ||
      !sym(h, "wc_priority_consensus_batch", batch_prio) || !sym(h, "wc_last_error", last_error) ||
      !sym(h, "wc_service_last_error", svc_last_error))
    return -1;
  wc_service* svc = nullptr;
  if (mode == 0) {
    const int rc = svc_create(device, 0, &svc);
    if (rc) return rc;
  }
  std::atomic<uint32_t> next{0};
  std::atomic<int> first_rc{0};
  auto worker = [&]() {
    wc_ctx* ctx = nullptr;
    if (mode == 1 && ctx_create(device, &ctx) != 0) {
      first_rc = 12;
      return;
    }
    for (;;) {
      const uint32_t i = next++;
      if (i >= n || first_rc.load()) break;
      const auto t0 = std::chrono::steady_clock::now();
      const int rc = mode == 0 ? svc_prio(svc, cfg, &loci[i], &results[i]) : batch_prio(ctx, cfg, 1, &loci[i], &results[i]);
      lat_ms[i] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      if (rc) {
        int z = 0;
        if (first_rc.compare_exchange_strong(z, rc))
          fprintf(stderr, "[api_bench] locus %u failed (rc %d): %s\n", i, rc, mode == 0 ? svc_last_error(svc) : last_error(ctx));
      }
    }
    if (ctx) ctx_destroy(ctx);
  };
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < threads; ++t) th.emplace_back(worker);
  for (auto& x : th) x.join();
  *wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (svc) {
    if (svc_stats) svc_stats_fn(svc, svc_stats);
    svc_destroy(svc);
  }
  return first_rc.load();
}
