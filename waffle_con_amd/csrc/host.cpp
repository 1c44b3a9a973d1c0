// C ABI of the waffle_con MI355X library (include/waffle_con.h).
//
// A batch uploads every problem's reads once into an HBM arena (wc_batch);
// each run launches the device-resident engine for the whole batch (one
// workgroup per problem, persistent grid pulling problems from an atomic
// counter, longest problems first; engine_host.cpp) and turns the device
// result records into the reference's result types (Consensus,
// DualConsensus, PriorityConsensus). Problems that outgrow a device capacity
// (wavefront length, node pool, consensus length, result records) are re-run
// on the device with larger capacities; no consensus work is ever done on the
// CPU.
#include <immintrin.h>
#include <atomic>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "host_internal.hpp"
#include "waffle_con_internal.hpp"

using namespace wc;
using namespace wch;

namespace wch {
std::string err_msg(int code) {
  switch (code) {
    case WC_E_FINALIZE_UNINIT: return "Finalize called on DWFA that was never initialized.";
    case WC_E_NO_START: return "Must have at least one initial offset of None to see the consensus.";
    case WC_E_COVERAGE_GAP: return "Encountered coverage gap";
    case WC_E_CAPACITY: return "Capacity is full";
    case WC_E_LOCKED: return "Consensus is locked, cannot modify";
    case WC_E_DUAL_TWICE: return "Cannot activate dual on a dual node";
    case WC_E_SAME_SYMBOL: return "Cannot activate dual mode with the same extension symbols";
    case WC_E_ROOT_INACTIVE: return "Root consensus node has no initially active sequences.";
    case WC_E_BAD_INPUT: return "invalid input";
    case WC_E_INVARIANT: return "internal invariant violated";
    case WC_E_LIMIT:
      return "device capacity limit exceeded (alphabet: more than 8 distinct symbols at one read's wavefront tips "
             "or 14 voted at one node side; or more than 64 children of one node)";
    case WC_E_HIP: return "HIP runtime failure";
    default: return "ok";
  }
}

// WC_E_LIMIT from an engine: what overflowed (engine_shared.hpp LIM_*)
std::string limit_msg(uint32_t why) {
  std::string m = "device capacity limit exceeded:";
  if (why & LIM_TIPS) m += " more than 8 distinct symbols at one read's wavefront tips;";
  if (why & LIM_VOTES) m += " more than 14 distinct symbols voted at one node side;";
  if (why & LIM_CHILDREN) m += " more than 64 children of one node;";
  if (why & LIM_OFFSET) m += " offset activation scratch (offset_window + offset_compare_length);";
  if (!(why & (LIM_TIPS | LIM_VOTES | LIM_CHILDREN | LIM_OFFSET))) return err_msg(WC_E_LIMIT);
  m.pop_back();
  return m;
}

// a problem still asking for more capacity after the last retry
std::string retry_msg(uint32_t st, uint32_t attempts) {
  std::string m = "device capacity limit exceeded: still too small after " + std::to_string(attempts) + " retries:";
  if (st & ST_RETRY_WCAP) m += " wavefront rows (edit distance);";
  if (st & ST_RETRY_PCAP) m += " node pool;";
  if (st & ST_RETRY_HEAP) m += " priority queue;";
  if (st & ST_RETRY_LCAP) m += " consensus length;";
  if (st & ST_RETRY_RMAX) m += " result records;";
  m.pop_back();
  return m;
}

int set_err(wc_ctx* ctx, int code, const std::string& msg) {
  if (ctx) ctx->err = msg;
  return code;
}

DevConfig to_dev(const wc_config& c) {
  DevConfig d;
  d.max_queue_size = c.max_queue_size;
  d.max_capacity_per_size = c.max_capacity_per_size;
  d.max_return_size = c.max_return_size;
  d.max_nodes_wo_constraint = c.max_nodes_wo_constraint;
  d.min_count = c.min_count;
  d.dual_max_ed_delta = c.dual_max_ed_delta;
  d.offset_window = c.offset_window;
  d.offset_compare_length = c.offset_compare_length;
  d.min_af = c.min_af;
  d.cost_mode = c.consensus_cost;
  d.wildcard = c.wildcard;
  d.weighted = c.weighted_by_ed;
  d.early = c.allow_early_termination;
  return d;
}

// ---- 2-bit packed uploads ----
// A batch whose reads use one four-symbol alphabet (the raw codes 0..3 of
// generate_test, or ASCII A/C/G/T) is packed on the host, 2 bits per base,
// while it is staged (the staging pass reads every byte anyway), crosses PCIe
// at a quarter of the bytes, and is expanded into the byte arena on the device
// (pack2.hip). Read r's packed bytes start at roff[r] / 4 (roff is 16-byte
// aligned); byte t holds bases 4t..4t+3, base 4t+k in bits 2k..2k+1; bases
// past the read's end pack as code 0 (the device writes zeros there).
namespace {
enum PackMode : int { kPackNone = 0, kPackRaw = 1, kPackAcgt = 2 };
// ASCII A/C/G/T -> (b >> 1) & 3 = 0, 1, 3, 2
inline int acgt_code(uint8_t x) {
  switch (x) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 3;
    case 'T': return 2;
    default: return -1;
  }
}
bool pack_read_scalar(const uint8_t* s, uint32_t from, uint32_t len, uint8_t* d, int mode) {
  const uint32_t padded = (len + 15) & ~15u;
  for (uint32_t i = from; i < padded; i += 4) {
    uint32_t b = 0;
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t pos = i + k;
      if (pos >= len) continue;
      const uint8_t x = s[pos];
      const int c = mode == kPackRaw ? (x < 4 ? (int)x : -1) : acgt_code(x);
      if (c < 0) return false;
      b |= (uint32_t)c << (2 * k);
    }
    d[i / 4] = (uint8_t)b;
  }
  return true;
}
// 64 bases -> 16 bytes per step: validate, map to codes, then two
// multiply-adds combine 4 codes into one byte and a truncation packs 16 of them
__attribute__((target("avx512f,avx512bw"))) bool pack_read_avx512(const uint8_t* s, uint32_t len, uint8_t* d,
                                                                   int mode) {
  uint32_t i = 0;
  const __m512i w16 = _mm512_set1_epi16(0x0401), w32 = _mm512_set1_epi32(0x00100001);
  for (; i + 64 <= len; i += 64) {
    const __m512i x = _mm512_loadu_si512((const void*)(s + i));
    __m512i c;
    if (mode == kPackRaw) {
      if (_mm512_test_epi8_mask(x, _mm512_set1_epi8((char)0xFC))) return false;
      c = x;
    } else {
      const __mmask64 ok = _mm512_cmpeq_epi8_mask(x, _mm512_set1_epi8('A')) |
                           _mm512_cmpeq_epi8_mask(x, _mm512_set1_epi8('C')) |
                           _mm512_cmpeq_epi8_mask(x, _mm512_set1_epi8('G')) |
                           _mm512_cmpeq_epi8_mask(x, _mm512_set1_epi8('T'));
      if (ok != ~0ull) return false;
      c = _mm512_and_si512(_mm512_srli_epi16(x, 1), _mm512_set1_epi8(3));
    }
    const __m512i t16 = _mm512_maddubs_epi16(c, w16);  // c0 + 4 c1
    const __m512i t32 = _mm512_madd_epi16(t16, w32);   // (c0 + 4 c1) + 16 (c2 + 4 c3)
    _mm_storeu_si128((__m128i*)(d + i / 4), _mm512_cvtepi32_epi8(t32));
  }
  return pack_read_scalar(s, i, len, d, mode);
}
bool have_avx512() {
  static const bool ok = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
  return ok;
}
}  // namespace

// Copies every read of `problems` into one 16-byte-aligned arena and uploads it.
// The host side is one pass of memcpy into pinned staging (split over threads
// by bytes), then a single DMA; the device buffer of `b` is reused when it is
// large enough (wc_batch_refill), so a refill needs no allocation.
// Transactional: the input is validated and the new read tables are built in
// locals first; a buffer that must grow is allocated next to the old one. `b`
// changes only when the whole upload succeeded. The one partial outcome is a
// failed copy into a reused buffer: the batch is then marked invalid and every
// later run on it returns WC_E_BAD_INPUT.
int upload_batch(wc_ctx* ctx, uint32_t n, const wc_problem* problems, wc_batch* b) {
  std::vector<BatchProblem> probs(n);
  uint64_t nr = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (problems[i].n_reads && (!problems[i].reads || !problems[i].lens))
      return set_err(ctx, WC_E_BAD_INPUT, "problem with reads but no read/length arrays");
    for (uint32_t r = 0; r < problems[i].n_reads; ++r) {
      if (problems[i].lens[r] >= (1ull << 31)) return set_err(ctx, WC_E_BAD_INPUT, "read longer than 2^31 bytes");
      if (problems[i].lens[r] && !problems[i].reads[r]) return set_err(ctx, WC_E_BAD_INPUT, "null read pointer");
    }
    nr += problems[i].n_reads;
  }
  std::vector<uint64_t> roff(nr, 0);
  std::vector<uint32_t> rlen(nr);
  std::vector<const uint8_t*> src(nr);
  uint64_t pos = 0, k = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const wc_problem& p = problems[i];
    BatchProblem& q = probs[i];
    q.read_begin = (uint32_t)k;
    q.n_reads = p.n_reads;
    q.offsets.assign(p.n_reads, -1);
    for (uint32_t r = 0; r < p.n_reads; ++r, ++k) {
      if (p.offsets) q.offsets[r] = p.offsets[r] < 0 ? -1 : p.offsets[r];
      roff[k] = pos;
      src[k] = p.reads[r];
      rlen[k] = (uint32_t)p.lens[r];
      pos += (p.lens[r] + 15) & ~15ull;
      q.max_len = std::max<uint32_t>(q.max_len, (uint32_t)p.lens[r]);
      q.work += p.lens[r];
    }
  }
  // reads start 16-byte aligned; 64 bytes of tail padding let the engine load
  // 64-byte windows with 16-byte accesses anywhere inside a read
  const uint64_t total = pos + 64;
  std::vector<uint8_t> fallback;
  uint8_t* h = nullptr;
  auto fill = [&](uint64_t r0, uint64_t r1) {
    for (uint64_t r = r0; r < r1; ++r) {
      const uint64_t len = rlen[r], pad = ((len + 15) & ~15ull) - len;
      if (len) memcpy(h + roff[r], src[r], len);
      if (pad) memset(h + roff[r] + len, 0, pad);
    }
  };
  // the alphabet of a packed upload, from the first read (the packer checks
  // every byte; one outside it sends the whole batch the byte way)
  int pmode = kPackNone;
  {
    const char* pe = getenv("WC_PACK");
    const bool want_pack = pe ? atoi(pe) != 0 : total >= (16ull << 20);
    for (uint64_t r = 0; want_pack && r < nr && pmode == kPackNone; ++r)
      if (rlen[r]) pmode = src[r][0] < 4 ? kPackRaw : (acgt_code(src[r][0]) >= 0 ? kPackAcgt : -1);
    if (pmode < 0) pmode = kPackNone;
  }
  const uint32_t plut = pmode == kPackRaw ? 0x03020100u : ('A' | 'C' << 8 | 'T' << 16 | (uint32_t)'G' << 24);
  ctx->last_upload_packed = 0;
  // device buffers: reused when large enough, else new ones beside the old
  DevBuf grown[3];
  DevBuf* dst[3] = {&b->reads, &b->roff, &b->rlen};
  const size_t want[3] = {total, std::max<size_t>(roff.size(), 1) * 8, std::max<size_t>(rlen.size(), 1) * 4};
  for (int i = 0; i < 3; ++i) {
    if (want[i] <= dst[i]->cap) continue;
    if (!grown[i].ensure(want[i])) {
      for (DevBuf& g : grown) g.release();
      return set_err(ctx, WC_E_HIP, "device allocation failed (reads)");
    }
    dst[i] = &grown[i];
  }
  const bool in_place = dst[0] == &b->reads || dst[1] == &b->roff || dst[2] == &b->rlen;
  if (in_place) b->valid = false;  // until every copy below has landed
  auto fail = [&](const std::string& what) {
    for (DevBuf& g : grown) g.release();
    return set_err(ctx, WC_E_HIP, what);
  };
  auto commit = [&]() {
    for (int i = 0; i < 3; ++i)
      if (dst[i] == &grown[i]) {
        DevBuf* old = i == 0 ? &b->reads : (i == 1 ? &b->roff : &b->rlen);
        old->release();
        *old = grown[i];
        grown[i].p = nullptr;
        grown[i].cap = 0;
      }
    b->ctx = ctx;
    b->probs.swap(probs);
    b->roff_h.swap(roff);
    b->rlen_h.swap(rlen);
    b->bytes = total;
    b->valid = true;
    return (int)WC_OK;
  };
  // staging threads: up to 16, or WC_UPLOAD_THREADS (a caller that computes
  // on another context while this one uploads may want to leave it cores)
  unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (const char* ut = getenv("WC_UPLOAD_THREADS")) hw = std::max(1, std::min(64, atoi(ut)));
  // reads split into contiguous ranges of about equal bytes, one per thread
  auto split_run = [&](uint64_t r_begin, uint64_t r_end, uint64_t nt, auto fn) {
    const uint64_t b0 = r_begin < nr ? roff[r_begin] : pos, b1 = r_end < nr ? roff[r_end] : pos;
    if (nt <= 1 || r_end - r_begin < 2) {
      fn(r_begin, r_end);
      return;
    }
    std::vector<std::thread> th;
    uint64_t r0 = r_begin;
    for (uint64_t t = 0; t < nt; ++t) {
      const uint64_t want_b = b0 + (b1 - b0) * (t + 1) / nt;
      uint64_t r1 = r0;
      while (r1 < r_end && (t + 1 == nt || roff[r1] < want_b)) ++r1;
      th.emplace_back(fn, r0, r1);
      r0 = r1;
    }
    for (auto& x : th) x.join();
  };
  // chunks of >= 64 MiB of reads (at most 8): the H2D copy of chunk k runs
  // while the host threads stage chunk k + 1; inside a chunk the reads are
  // split into contiguous ranges of about equal bytes, one per thread (>= 8 MiB
  // each). Packed: every read is packed straight from the caller's buffer into
  // pinned staging (AVX-512 where the CPU has it) and a quarter of the bytes
  // crosses PCIe into ctx->upk; a byte outside the alphabet stops it and the
  // whole batch goes again the byte way.
  bool packed = pmode != kPackNone && ctx->upstage.ensure(pos / 4 + 16) && ctx->upk.ensure(pos / 4 + 16);
  const bool simd = have_avx512() && !getenv("WC_PACK_SCALAR");  // (test hook: the scalar packer)
  std::atomic<bool> ok{true};
  auto pack = [&](uint64_t r0, uint64_t r1) {
    uint8_t* hp = (uint8_t*)ctx->upstage.p;
    for (uint64_t r = r0; r < r1 && ok.load(std::memory_order_relaxed); ++r) {
      const bool good = simd ? pack_read_avx512(src[r], rlen[r], hp + roff[r] / 4, pmode)
                             : pack_read_scalar(src[r], 0, rlen[r], hp + roff[r] / 4, pmode);
      if (!good) ok.store(false, std::memory_order_relaxed);
    }
  };
  // (test hooks: WC_UPLOAD_CHUNK_SHIFT / WC_UPLOAD_THREAD_SHIFT shrink the
  // 64 MiB chunks and the 8 MiB per staging thread, so small batches run the
  // multi-chunk, multi-thread path)
  const char* cse = getenv("WC_UPLOAD_CHUNK_SHIFT");
  const char* tse = getenv("WC_UPLOAD_THREAD_SHIFT");
  const int cshift = cse ? std::max(4, std::min(40, atoi(cse))) : 26;
  const int tshift = tse ? std::max(4, std::min(40, atoi(tse))) : 23;
  const uint64_t nch = std::max<uint64_t>(1, std::min<uint64_t>(8, total >> cshift));
  for (int pass = packed ? 0 : 1; pass < 2; ++pass) {
    const bool pk = pass == 0;
    if (!pk) {
      // staging of the byte path (after a packed attempt's copies have drained)
      if (hipStreamSynchronize(ctx->stream) != hipSuccess) return fail("read upload failed");
      if (!ctx->upstage.ensure(total)) {
        fallback.resize(total);
        h = fallback.data();
      } else {
        h = (uint8_t*)ctx->upstage.p;
      }
    }
    uint64_t c_r0 = 0;
    for (uint64_t c = 0; c < nch && (!pk || ok.load()); ++c) {
      const uint64_t want_end = pos * (c + 1) / nch;
      uint64_t c_r1 = c_r0;
      while (c_r1 < nr && (c + 1 == nch || roff[c_r1] < want_end)) ++c_r1;
      const uint64_t b0 = c_r0 < nr ? roff[c_r0] : pos;
      const uint64_t b1 = c_r1 < nr ? roff[c_r1] : pos;
      const uint64_t nt = std::max<uint64_t>(1, std::min<uint64_t>(hw, (b1 - b0) >> tshift));
      const bool last = c + 1 == nch;
      if (pk) {
        split_run(c_r0, c_r1, nt, pack);
        if (!ok.load()) break;
        if (b1 > b0 && hipMemcpyAsync((uint8_t*)ctx->upk.p + b0 / 4, (uint8_t*)ctx->upstage.p + b0 / 4, (b1 - b0) / 4,
                                      hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
          return fail("read upload failed");
      } else {
        split_run(c_r0, c_r1, nt, fill);
        if (last) memset(h + pos, 0, 64);
        const uint64_t e1 = last ? total : b1;
        if (e1 > b0 && hipMemcpyAsync((uint8_t*)dst[0]->p + b0, h + b0, e1 - b0, hipMemcpyHostToDevice,
                                      ctx->stream) != hipSuccess)
          return fail("read upload failed");
      }
      c_r0 = c_r1;
    }
    if (pk && !ok.load()) continue;  // a byte outside the alphabet
    packed = pk;
    break;
  }
  if (!roff.empty() &&
      hipMemcpyAsync(dst[1]->p, roff.data(), roff.size() * 8, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
    return fail("read table upload failed");
  if (!rlen.empty() &&
      hipMemcpyAsync(dst[2]->p, rlen.data(), rlen.size() * 4, hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
    return fail("read table upload failed");
  if (packed) {
    launch_unpack2((const uint32_t*)ctx->upk.p, (const uint64_t*)dst[1]->p, (const uint32_t*)dst[2]->p, (uint32_t)nr,
                   plut, (uint8_t*)dst[0]->p, pos, ctx->stream);
    if (hipGetLastError() != hipSuccess) return fail("read upload failed (device unpack)");
  }
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return fail("read upload failed");
  ctx->last_upload_packed = packed ? pos / 4 : 0;
  return commit();
}

}  // namespace wch

namespace {
// ConsensusDWFA / DualConsensusDWFA over every problem of a resident batch
int batch_run(wc_ctx* ctx, wc_batch* b, const wc_config& cfg, uint32_t sides, wc_results* R) {
  auto t0 = std::chrono::steady_clock::now();
  const uint32_t n = (uint32_t)b->probs.size();
  R->kind = sides == 1 ? 0 : 1;
  R->probs.resize(n);
  std::vector<SubProb> items(n);
  std::vector<EngineOut> outs(n);
  for (uint32_t i = 0; i < n; ++i) {
    const BatchProblem& q = b->probs[i];
    SubProb& s = items[i];
    s.gid.resize(q.n_reads);
    std::iota(s.gid.begin(), s.gid.end(), q.read_begin);
    s.max_len = q.max_len;
    s.work = q.work;
    const int rc = activation_plan(cfg, q.offsets, s, outs[i].error);
    if (rc != WC_OK) outs[i].status = rc;
  }
  double kms = 0;
  uint64_t nl = 0;
  const auto t1 = std::chrono::steady_clock::now();
  std::vector<uint8_t> built(n, 0);
  if (sides == 1) {
    uint64_t guess = 0;
    for (uint32_t i = 0; i < n; ++i) guess += b->probs[i].max_len + b->probs[i].max_len / 16;
    R->a_seq.reserve(guess);
    R->p_seq0.assign(n, ~0ull);
    R->p_sc0.assign(n, ~0ull);
  }
  const std::function<void(uint32_t)> build = [&](uint32_t i) {
    R->probs[i].done_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (sides == 1) {
      build_single(outs[i], cfg.consensus_cost, R->probs[i]);
      pack_single(R, i);
    } else {
      build_dual(outs[i], b->probs[i].n_reads, cfg.consensus_cost, R->probs[i]);
    }
    built[i] = 1;
  };
  int rc = run_engine(ctx, b, cfg, sides, items, outs, kms, nl, &build);
  if (rc != WC_OK) return rc;
  const auto t2 = std::chrono::steady_clock::now();
  for (uint32_t i = 0; i < n; ++i)
    if (!built[i]) build(i);
  double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (getenv("WC_HOST_TIMING")) {
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point z) {
      return std::chrono::duration<double, std::milli>(z - a).count();
    };
    fprintf(stderr, "[wc] host: plan %.3f ms, engine %.3f ms (kernel %.3f), results %.3f ms\n", ms(t0, t1), ms(t1, t2),
            kms, ms(t2, std::chrono::steady_clock::now()));
  }
  fill_stats(R, kms, nl, wall);
  return WC_OK;
}

template <class F>
int with_batch(wc_ctx* ctx, uint32_t n, const wc_problem* problems, F&& fn) {
  std::unique_ptr<wc_batch> b(new wc_batch());
  int rc = upload_batch(ctx, n, problems, b.get());
  if (rc != WC_OK) return rc;
  return fn(b.get());
}
}  // namespace

// ------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------
extern "C" {

void wc_config_default(wc_config* c) {
  memset(c, 0, sizeof(*c));
  c->consensus_cost = 0;
  c->wildcard = -1;
  c->max_queue_size = 20;
  c->max_capacity_per_size = 20;
  c->max_return_size = 10;
  c->max_nodes_wo_constraint = 1000;
  c->min_count = 3;
  c->min_af = 0.0;
  c->dual_max_ed_delta = 20;
  c->offset_window = 50;
  c->offset_compare_length = 50;
  c->weighted_by_ed = 0;
  c->allow_early_termination = 0;
  c->auto_shift_offsets = 1;
}

int wc_ctx_create(int device, wc_ctx** out) {
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return WC_E_HIP;
  if (device < 0 || device >= ndev) return WC_E_HIP;
  if (hipSetDevice(device) != hipSuccess) return WC_E_HIP;
  wc_ctx* ctx = new wc_ctx();
  ctx->device = device;
  hipDeviceProp_t prop;
  if (const char* e = getenv("WC_DEVICE_SHARE")) ctx->share = std::max(1, atoi(e));
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->n_cu = prop.multiProcessorCount;
  // co-tenants of one device (WC_DEVICE_SHARE = k processes): every launch of
  // this context is planned for 1/k of the CUs, so k persistent launches fit
  // side by side instead of each asking for the whole chip
  ctx->n_cu = std::max(1, ctx->n_cu / ctx->share);
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess) {
    delete ctx;
    return WC_E_HIP;
  }
  *out = ctx;
  return WC_OK;
}

void wc_ctx_destroy(wc_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  destroy_launches(ctx);
  ctx->jobs.release();
  ctx->upstage.release();
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* wc_last_error(const wc_ctx* ctx) { return ctx ? ctx->err.c_str() : "no context"; }

uint32_t wc_engines_used(wc_ctx* ctx, int reset) {
  if (!ctx) return 0;
  return reset ? ctx->engines_used.exchange(0) : ctx->engines_used.load();
}

const char* wc_engine_name(uint32_t bit) { return bit < wch::kNumEngineNames ? wch::kEngineNames[bit] : nullptr; }

uint64_t wc_last_upload_packed(const wc_ctx* ctx) { return ctx ? ctx->last_upload_packed : 0; }

int wc_batch_create(wc_ctx* ctx, uint32_t n, const wc_problem* problems, wc_batch** out) {
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  std::unique_ptr<wc_batch> b(new wc_batch());
  int rc = upload_batch(ctx, n, problems, b.get());
  if (rc != WC_OK) return rc;
  *out = b.release();
  return WC_OK;
}

int wc_batch_refill(wc_ctx* ctx, wc_batch* b, uint32_t n, const wc_problem* problems) {
  if (!b) return set_err(ctx, WC_E_BAD_INPUT, "null batch");
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  return upload_batch(ctx, n, problems, b);
}

void wc_batch_free(wc_batch* b) { delete b; }

uint64_t wc_batch_bytes(const wc_batch* b) { return b ? b->bytes : 0; }

int wc_batch_consensus(wc_ctx* ctx, wc_batch* b, const wc_config* cfg, wc_results** out) {
  *out = nullptr;
  if (!b || !b->valid) return set_err(ctx, WC_E_BAD_INPUT, "batch is not usable (a failed refill left it incomplete)");
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  std::unique_ptr<wc_results> R(new wc_results());
  int rc = batch_run(ctx, b, *cfg, 1, R.get());
  if (rc != WC_OK) return rc;
  *out = R.release();
  return WC_OK;
}

int wc_batch_dual_consensus(wc_ctx* ctx, wc_batch* b, const wc_config* cfg, wc_results** out) {
  *out = nullptr;
  if (!b || !b->valid) return set_err(ctx, WC_E_BAD_INPUT, "batch is not usable (a failed refill left it incomplete)");
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  std::unique_ptr<wc_results> R(new wc_results());
  int rc = batch_run(ctx, b, *cfg, 2, R.get());
  if (rc != WC_OK) return rc;
  *out = R.release();
  return WC_OK;
}

int wc_consensus_batch(wc_ctx* ctx, const wc_config* cfg, uint32_t n, const wc_problem* problems, wc_results** out) {
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  return with_batch(ctx, n, problems, [&](wc_batch* b) { return wc_batch_consensus(ctx, b, cfg, out); });
}

int wc_dual_consensus_batch(wc_ctx* ctx, const wc_config* cfg, uint32_t n, const wc_problem* problems,
                            wc_results** out) {
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  return with_batch(ctx, n, problems, [&](wc_batch* b) { return wc_batch_dual_consensus(ctx, b, cfg, out); });
}

// ---- PriorityConsensusDWFA (priority_consensus.rs:172-341) ----
// Each problem keeps the reference's LIFO work stack; every sub-problem is a
// DualConsensusDWFA run on the device, streamed through up to two concurrent
// engine launches (engine_host.cpp priority_stream).
int wc_priority_consensus_batch(wc_ctx* ctx, const wc_config* cfg, uint32_t n, const wc_chain_problem* problems,
                                wc_results** out) {
  auto t0 = std::chrono::steady_clock::now();
  *out = nullptr;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  std::unique_ptr<wc_results> R(new wc_results());
  R->kind = 2;
  int rc = priority_stream(ctx, *cfg, n, problems, R.get());
  if (rc != WC_OK) return rc;
  const double kms = R->stats.kernel_ms;
  const uint64_t nl = R->stats.launches;
  double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  fill_stats(R.get(), kms, nl, wall);
  *out = R.release();
  return WC_OK;
}

void wc_results_free(wc_results* r) { delete r; }
uint32_t wc_results_problems(const wc_results* r) { return (uint32_t)r->probs.size(); }
int wc_results_status(const wc_results* r, uint32_t p) { return p < r->probs.size() ? r->probs[p].status : WC_E_BAD_INPUT; }
const char* wc_results_error(const wc_results* r, uint32_t p) {
  return p < r->probs.size() ? r->probs[p].error.c_str() : "no such problem";
}
uint32_t wc_results_count(const wc_results* r, uint32_t p) {
  if (p >= r->probs.size()) return 0;
  const ProbRes& q = r->probs[p];
  if (r->kind == 0) return (uint32_t)q.single.size();
  if (r->kind == 1) return (uint32_t)q.dual.size();
  return (uint32_t)q.chains.size();
}

int wc_results_single(const wc_results* r, uint32_t p, uint32_t k, const uint8_t** seq, uint64_t* seq_len,
                      const uint64_t** scores, uint64_t* n_scores) {
  if (r->kind != 0 || p >= r->probs.size() || k >= r->probs[p].single.size()) return WC_E_BAD_INPUT;
  const ConsRec& c = r->probs[p].single[k];
  *seq = c.seq.data();
  *seq_len = c.seq.size();
  *scores = c.scores.data();
  *n_scores = c.scores.size();
  return WC_OK;
}

int wc_results_single_sizes(const wc_results* r, uint64_t* n_results, uint64_t* seq_bytes, uint64_t* n_scores) {
  if (r->kind != 0) return WC_E_BAD_INPUT;
  uint64_t nr = 0, sb = 0, ns = 0;
  for (const ProbRes& p : r->probs)
    for (const ConsRec& c : p.single) {
      nr++;
      sb += c.seq.size();
      ns += c.scores.size();
    }
  *n_results = nr;
  *seq_bytes = sb;
  *n_scores = ns;
  return WC_OK;
}

int wc_results_single_pack(const wc_results* r, int32_t* status, uint32_t* count, uint8_t* seq, uint64_t* seq_off,
                           uint64_t* scores, uint64_t* score_off) {
  if (r->kind != 0) return WC_E_BAD_INPUT;
  uint64_t k = 0, so = 0, co = 0;
  seq_off[0] = score_off[0] = 0;
  for (size_t p = 0; p < r->probs.size(); ++p) {
    const ProbRes& pr = r->probs[p];
    status[p] = pr.status;
    count[p] = (uint32_t)pr.single.size();
    for (const ConsRec& c : pr.single) {
      if (!c.seq.empty()) memcpy(seq + so, c.seq.data(), c.seq.size());
      if (!c.scores.empty()) memcpy(scores + co, c.scores.data(), c.scores.size() * 8);
      so += c.seq.size();
      co += c.scores.size();
      seq_off[++k] = so;
      score_off[k] = co;
    }
  }
  return WC_OK;
}

int wc_results_single_view(wc_results* r, const int32_t** status, const uint32_t** count, const uint8_t** seq,
                           const uint64_t** scores, const uint64_t** index) {
  if (r->kind != 0) return WC_E_BAD_INPUT;
  if (!r->view_ready) {
    const uint32_t n = (uint32_t)r->probs.size();
    if (r->p_seq0.size() != n) {
      r->p_seq0.assign(n, ~0ull);
      r->p_sc0.assign(n, ~0ull);
    }
    for (uint32_t p = 0; p < n; ++p)
      if (r->p_seq0[p] == ~0ull) pack_single(r, p);
    r->v_status.resize(std::max<size_t>(n, 1));
    r->v_count.resize(std::max<size_t>(n, 1));
    r->v_idx.clear();
    for (uint32_t p = 0; p < n; ++p) {
      const ProbRes& pr = r->probs[p];
      r->v_status[p] = pr.status;
      r->v_count[p] = (uint32_t)pr.single.size();
      uint64_t so = r->p_seq0[p], co = r->p_sc0[p];
      for (const ConsRec& c : pr.single) {
        r->v_idx.insert(r->v_idx.end(), {so, (uint64_t)c.seq.size(), co, (uint64_t)c.scores.size()});
        so += c.seq.size();
        co += c.scores.size();
      }
    }
    if (r->a_seq.empty()) r->a_seq.push_back(0);
    if (r->a_sc.empty()) r->a_sc.push_back(0);
    if (r->v_idx.empty()) r->v_idx.push_back(0);
    r->view_ready = true;
  }
  *status = r->v_status.data();
  *count = r->v_count.data();
  *seq = r->a_seq.data();
  *scores = r->a_sc.data();
  *index = r->v_idx.data();
  return WC_OK;
}

int wc_results_dual(const wc_results* r, uint32_t p, uint32_t k, wc_dual_view* o) {
  if (r->kind != 1 || p >= r->probs.size() || k >= r->probs[p].dual.size()) return WC_E_BAD_INPUT;
  const DualRec& d = r->probs[p].dual[k];
  o->seq1 = d.c1.seq.data();
  o->len1 = d.c1.seq.size();
  o->scores_c1 = d.c1.scores.data();
  o->n_scores_c1 = d.c1.scores.size();
  o->has_c2 = d.has_c2;
  o->seq2 = d.c2.seq.data();
  o->len2 = d.c2.seq.size();
  o->scores_c2 = d.c2.scores.data();
  o->n_scores_c2 = d.c2.scores.size();
  o->is_consensus1 = d.is_c1.data();
  o->scores1 = d.s1.data();
  o->scores2 = d.s2.data();
  o->n_reads = d.is_c1.size();
  return WC_OK;
}

uint32_t wc_results_chain_len(const wc_results* r, uint32_t p, uint32_t k) {
  if (r->kind != 2 || p >= r->probs.size() || k >= r->probs[p].chains.size()) return 0;
  return (uint32_t)r->probs[p].chains[k].size();
}

int wc_results_chain(const wc_results* r, uint32_t p, uint32_t k, uint32_t level, const uint8_t** seq,
                     uint64_t* seq_len, const uint64_t** scores, uint64_t* n_scores) {
  if (r->kind != 2 || p >= r->probs.size() || k >= r->probs[p].chains.size() ||
      level >= r->probs[p].chains[k].size())
    return WC_E_BAD_INPUT;
  const ConsRec& c = r->probs[p].chains[k][level];
  *seq = c.seq.data();
  *seq_len = c.seq.size();
  *scores = c.scores.data();
  *n_scores = c.scores.size();
  return WC_OK;
}

int wc_results_sequence_indices(const wc_results* r, uint32_t p, const uint64_t** idx, uint64_t* n) {
  if (r->kind != 2 || p >= r->probs.size()) return WC_E_BAD_INPUT;
  *idx = r->probs[p].indices.data();
  *n = r->probs[p].indices.size();
  return WC_OK;
}

int wc_results_stats(const wc_results* r, wc_stats* out) {
  *out = r->stats;
  return WC_OK;
}

int wc_results_problem_stats(const wc_results* r, uint32_t p, wc_stats* o) {
  if (p >= r->probs.size()) return WC_E_BAD_INPUT;
  memset(o, 0, sizeof(*o));
  const uint64_t* s = r->probs[p].stats;
  o->updates = s[S_UPDATES];
  o->w_out = s[S_WOUT];
  o->compares = s[S_COMPARES];
  o->ed_increases = s[S_EDINC];
  o->finalizes = s[S_FINALIZES];
  o->pops = s[S_POPS];
  o->nodes_explored = s[S_EXPLORED];
  o->nodes_ignored = s[S_IGNORED];
  o->peak_queue_size = s[S_PEAKQ];
  o->row_bytes = s[S_ROWB];
  o->wall_ms = r->probs[p].done_ms;
  o->start_ms = r->probs[p].start_ms;
  return WC_OK;
}

// ---- standalone DWFALite batch (dynamic_wfa.rs:48-265) ----
int wc_dwfa_batch(wc_ctx* ctx, uint32_t n, wc_dwfa_job* jobs) {
  if (n == 0) return WC_OK;
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  // one arena: per job baseline | other | wavefront (u32, cap)
  std::vector<uint64_t> boff(n), ooff(n), woff(n);
  uint64_t total = 0;
  for (uint32_t i = 0; i < n; ++i) {
    if (jobs[i].wf_cap < jobs[i].wf_len || jobs[i].wf_len != 2 * jobs[i].e + 1)
      return set_err(ctx, WC_E_BAD_INPUT, "wavefront length must be 2e+1 and fit wf_cap");
    boff[i] = total;
    total += (jobs[i].baseline_len + 15) & ~15ull;
    ooff[i] = total;
    total += (jobs[i].other_len + 15) & ~15ull;
    woff[i] = total;
    total += (jobs[i].wf_cap * 4 + 15) & ~15ull;
  }
  // reads start 16-byte aligned; 64 bytes of tail padding let the engine load
  // 64-byte windows with 16-byte accesses anywhere inside a read
  std::vector<uint8_t> h(total + 64);
  std::vector<DwfaDevJob> dj(n);
  for (uint32_t i = 0; i < n; ++i) {
    const wc_dwfa_job& j = jobs[i];
    if (j.baseline_len) memcpy(h.data() + boff[i], j.baseline, j.baseline_len);
    if (j.other_len) memcpy(h.data() + ooff[i], j.other, j.other_len);
    uint32_t* wf = (uint32_t*)(h.data() + woff[i]);
    for (uint64_t k = 0; k < j.wf_len; ++k) wf[k] = (uint32_t)j.wavefront[k];
  }
  DevBuf arena;
  if (!arena.ensure(h.size()) || !ctx->jobs.ensure(n * sizeof(DwfaDevJob)))
    return set_err(ctx, WC_E_HIP, "device allocation failed (dwfa)");
  uint8_t* base = (uint8_t*)arena.p;
  for (uint32_t i = 0; i < n; ++i) {
    const wc_dwfa_job& j = jobs[i];
    DwfaDevJob& d = dj[i];
    memset(&d, 0, sizeof(d));
    d.baseline = base + boff[i];
    d.blen = (uint32_t)j.baseline_len;
    d.other = base + ooff[i];
    d.olen = (uint32_t)j.other_len;
    d.offset = (uint32_t)j.offset;
    d.wildcard = j.wildcard;
    d.early = j.early;
    d.op = j.op;
    d.e = (uint32_t)j.e;
    d.wf = (uint32_t*)(base + woff[i]);
    d.wf_cap = (uint32_t)j.wf_cap;
  }
  int rc = WC_OK;
  do {
    if (hipMemcpyAsync(arena.p, h.data(), h.size(), hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
        hipMemcpyAsync(ctx->jobs.p, dj.data(), n * sizeof(DwfaDevJob), hipMemcpyHostToDevice, ctx->stream) !=
            hipSuccess) {
      rc = set_err(ctx, WC_E_HIP, "copy to device failed (dwfa)");
      break;
    }
    launch_dwfa_jobs((DwfaDevJob*)ctx->jobs.p, n, ctx->stream);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(ctx->stream) != hipSuccess ||
        hipMemcpy(dj.data(), ctx->jobs.p, n * sizeof(DwfaDevJob), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(h.data(), arena.p, h.size(), hipMemcpyDeviceToHost) != hipSuccess) {
      rc = set_err(ctx, WC_E_HIP, "dwfa kernel failed");
      break;
    }
    for (uint32_t i = 0; i < n; ++i) {
      wc_dwfa_job& j = jobs[i];
      const DwfaDevJob& d = dj[i];
      j.status = (int32_t)d.status;
      if (d.status != 0) continue;
      j.e = d.e;
      const uint32_t W = 2 * d.e + 1;
      j.wf_len = W;
      const uint32_t* wf = (const uint32_t*)(h.data() + woff[i]);
      for (uint32_t k = 0; k < W && k < j.wf_cap; ++k) j.wavefront[k] = wf[k];
      j.n_cand = d.n_cand;
      for (uint32_t k = 0; k < d.n_cand && k < 16; ++k) {
        j.cand_syms[k] = d.cand_syms[k];
        j.cand_counts[k] = d.cand_counts[k];
        j.cand_first[k] = d.cand_first[k];
      }
    }
  } while (0);
  arena.release();
  return rc;
}

// ---- batched wfa_ed_config (sequence_alignment.rs:18-87) ----
// Pairs go to the device in launches whose sequence arena + scratch rows stay
// under kEdLaunchBytes (a single larger pair gets a launch of its own).
int wc_wfa_ed_batch(wc_ctx* ctx, uint32_t n, const uint8_t* const* v1, const uint64_t* l1, const uint8_t* const* v2,
                    const uint64_t* l2, uint8_t require_both_end, int32_t wildcard, uint64_t* out_ed) {
  if (n == 0) return WC_OK;
  if (!v1 || !l1 || !v2 || !l2 || !out_ed) return set_err(ctx, WC_E_BAD_INPUT, "wc_wfa_ed_batch: null argument");
  for (uint32_t i = 0; i < n; ++i) {
    if (l1[i] >= (1ull << 31) || l2[i] >= (1ull << 31))
      return set_err(ctx, WC_E_BAD_INPUT, "wc_wfa_ed_batch: sequence length must be < 2^31");
    if ((l1[i] && !v1[i]) || (l2[i] && !v2[i])) return set_err(ctx, WC_E_BAD_INPUT, "wc_wfa_ed_batch: null sequence");
  }
  if (hipSetDevice(ctx->device) != hipSuccess) return set_err(ctx, WC_E_HIP, "hipSetDevice failed");
  constexpr uint64_t kEdLaunchBytes = 1ull << 30;
  auto a16 = [](uint64_t x) { return (x + 15) & ~15ull; };
  auto cap_of = [&](uint32_t i) { return 2 * (l1[i] + l2[i]) + 3; };
  DevBuf arena, scratch, jobs, out;
  int rc = WC_OK;
  for (uint32_t b = 0; b < n && rc == WC_OK;) {
    // [b, e): pairs of this launch
    uint32_t e = b;
    uint64_t sbytes = 0, sents = 0;
    while (e < n) {
      const uint64_t add = a16(l1[e]) + a16(l2[e]), ents = 2 * cap_of(e);
      if (e > b && sbytes + add + 8 * (sents + ents) > kEdLaunchBytes) break;
      sbytes += add;
      sents += ents;
      ++e;
    }
    const uint32_t m = e - b;
    std::vector<uint8_t> h(sbytes + 16);
    std::vector<EdDevJob> dj(m);
    uint64_t so = 0, eo = 0;
    for (uint32_t k = 0; k < m; ++k) {
      const uint32_t i = b + k;
      EdDevJob& d = dj[k];
      d.v1_off = so;
      if (l1[i]) memcpy(h.data() + so, v1[i], l1[i]);
      so += a16(l1[i]);
      d.v2_off = so;
      if (l2[i]) memcpy(h.data() + so, v2[i], l2[i]);
      so += a16(l2[i]);
      d.l1 = (uint32_t)l1[i];
      d.l2 = (uint32_t)l2[i];
      d.cap = cap_of(i);
      d.scr_off = eo;
      eo += 2 * d.cap;
    }
    if (!arena.ensure(h.size()) || !scratch.ensure(8 * eo) || !jobs.ensure(m * sizeof(EdDevJob)) ||
        !out.ensure(8ull * m)) {
      rc = set_err(ctx, WC_E_HIP, "device allocation failed (wfa_ed batch)");
      break;
    }
    if (hipMemcpyAsync(arena.p, h.data(), h.size(), hipMemcpyHostToDevice, ctx->stream) != hipSuccess ||
        hipMemcpyAsync(jobs.p, dj.data(), m * sizeof(EdDevJob), hipMemcpyHostToDevice, ctx->stream) != hipSuccess) {
      rc = set_err(ctx, WC_E_HIP, "copy to device failed (wfa_ed batch)");
      break;
    }
    launch_wfa_ed_batch((const EdDevJob*)jobs.p, m, (const uint8_t*)arena.p, (uint64_t*)scratch.p, (int)wildcard,
                        require_both_end ? 1u : 0u, (uint64_t*)out.p, ctx->stream);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(out_ed + b, out.p, 8ull * m, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
        hipStreamSynchronize(ctx->stream) != hipSuccess) {
      rc = set_err(ctx, WC_E_HIP, "wfa_ed kernel failed");
      break;
    }
    for (uint32_t k = 0; k < m; ++k)
      if (out_ed[b + k] == ~0ull) {
        rc = set_err(ctx, WC_E_LIMIT, "wfa_ed scratch row too short");
        break;
      }
    b = e;
  }
  arena.release();
  scratch.release();
  jobs.release();
  out.release();
  return rc;
}

// ---- generator ----
struct wc_gen {
  std::vector<uint8_t> consensus;
  std::vector<std::vector<uint8_t>> samples;
};

int wc_generate_test(uint8_t alphabet, uint64_t seq_len, uint64_t num_samples, double error_rate, uint64_t seed,
                     wc_gen** handle) {
  if (alphabet < 2 || !(error_rate >= 0.0 && error_rate <= 1.0)) return WC_E_BAD_INPUT;
  wc_gen* g = new wc_gen();
  wc::generate_test(alphabet, seq_len, num_samples, error_rate, seed, g->consensus, g->samples);
  *handle = g;
  return WC_OK;
}
const uint8_t* wc_gen_consensus(const wc_gen* g, uint64_t* len) {
  *len = g->consensus.size();
  return g->consensus.data();
}
const uint8_t* wc_gen_sample(const wc_gen* g, uint64_t i, uint64_t* len) {
  if (i >= g->samples.size()) {
    *len = 0;
    return nullptr;
  }
  *len = g->samples[i].size();
  return g->samples[i].data();
}
void wc_gen_free(wc_gen* g) { delete g; }

}  // extern "C"
