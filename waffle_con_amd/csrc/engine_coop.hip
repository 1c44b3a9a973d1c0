// The one-wave dual engine's search on several cooperating waves (namespace
// wcc, wave_dual.hip.hpp with kCoop): a workgroup of kEW waves per problem,
// wave w's lane l holding read 64 w + l, for dual searches without offsets of
// 65-256 reads in launches whose latency is what counts (few problems: a
// PriorityConsensusDWFA call on one locus, cfg4; a deep cfg5 locus alone).
// The single-wave engine runs such problems two reads per lane (65-128
// reads) or not at all, and the block engines' per-pop serial sections sit
// between barriers of every wave. Here the per-read phases of a pop (the hot
// state, the analysis, the push, prune and cost) run on every wave, one read
// per lane; every wave keeps the search control in registers and computes it
// from the same exchanged values (the nominations, flags and cost partials
// through LDS), and wave 0 alone writes the shared state (heap, trackers,
// free stack, slot metadata). Same source as engine.hip.
#define WC_WAVE_DUAL 1
#define WC_COOP 1
#define WC_DUAL_ONLY 1
#define WC_ENGINE_NS wcc
#define WC_BLOCK 256
// (waves per SIMD the build is compiled for: WC_COOP_WPE. Its launches hold
// at most one problem per CU, so the default is 1: 512 registers with the
// AGPRs and no VGPR spills (37 at 2); 7527s 78-read level 10.5 -> 9.9 us per
// pop, cfg4s 100-read group 13.6 -> 12.7, gpurun_out/r06cd*)
#ifndef WC_COOP_WPE
#define WC_COOP_WPE 1
#endif
#define WC_WAVES_PER_EU WC_COOP_WPE
#define WC_DUAL_WAVES_PER_EU WC_COOP_WPE
#define WC_WAVE2_WPE WC_COOP_WPE
#include "engine.hip"
