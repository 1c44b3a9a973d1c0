// The cooperative wave build on 2 waves (namespace wcc2, engine_coop.hip's
// search with 128-thread workgroups): problems of 65-128 reads, where the
// 4-wave build would carry two idle waves through every barrier and its votes
// over four nomination arrays instead of two.
#define WC_WAVE_DUAL 1
#define WC_COOP 1
#define WC_DUAL_ONLY 1
#define WC_ENGINE_NS wcc2
#define WC_BLOCK 128
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
