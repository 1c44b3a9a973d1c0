// The single engine with 1024-thread workgroups (16 x wave64, namespace wcu),
// for batch launches of at most one problem per CU (a single deep locus, a
// handful of loci): the whole CU works on one problem. The chain walk deals
// a 100-read locus over 16 waves (6-7 reads each instead of 25), so each
// wave's edit-distance increases, which it runs one read at a time, shrink
// by the same factor, and the 4 waves per SIMD hide each other's memory
// latency. 128 VGPRs per lane (16 waves on 4 SIMDs). Same source as
// engine.hip; the per-wave parts of the layouts are sized for 16 waves
// (engine_shared.hpp chain_lds_bytes / act_scr_u64, Caps::waves).
// (WC_CU_BLOCK / WC_CU_WPE: experiment builds, e.g. 512 threads at 2
// waves per SIMD with the grouped increases, -DWC_GROUP_HEAVY)
#define WC_CU 1
#define WC_SINGLE_ONLY 1
#define WC_ENGINE_NS wcu
#ifndef WC_CU_BLOCK
#define WC_CU_BLOCK 1024
#endif
#ifndef WC_CU_WPE
#define WC_CU_WPE 4
#endif
#define WC_BLOCK WC_CU_BLOCK
#define WC_WAVES_PER_EU WC_CU_WPE
#include "engine.hip"
