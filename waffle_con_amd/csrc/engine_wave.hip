// The dual engine on one wave per problem (namespace wcw, wave_dual.hip.hpp):
// lane r holds read r (and r + 64), the popped node's per-read state stays in
// LDS across pops and the tip bytes of its frontier in registers, so the
// common pop (the previous pop's in-place child) makes no dependent HBM round
// trip. For dual searches without offsets of at most 128 reads (the
// PriorityConsensusDWFA sub-problems of cfg5). Same source as engine.hip.
#define WC_WAVE_DUAL 1
#define WC_DUAL_ONLY 1
#define WC_ENGINE_NS wcw
#define WC_BLOCK 64
#define WC_WAVES_PER_EU 2
// waves per SIMD the wave kernels are built for. The two-reads-per-lane
// kernel (launches with problems of 65-128 reads: cfg5 batches) at 1: 512
// registers with the AGPRs and no VGPR spills (226 at 2); an 80-read
// sub-problem alone 21.4 -> 17.2 us/pop, the 10,000-locus cfg5 batch 323 ->
// 361 loci/s, the 2,000-locus one 19.0 -> 15.8 s, despite half the
// workgroups per CU. The one-read-per-lane kernel keeps 2 (5949's full-read
// level alone: 12.0 us/pop at either). Re-measured at the end of round 5
// (133 VGPRs spilled at 2, none at 1): 80-read sub-problem 12.0 (1) vs 15.0
// (2) us/pop, the 10,000-locus batch 19.8 vs 24.1 s (gpurun_out/r05wpe).
// WC_WAVE_WPE=<k> builds both at k.
#ifdef WC_WAVE_WPE
#define WC_DUAL_WAVES_PER_EU WC_WAVE_WPE
#define WC_WAVE2_WPE WC_WAVE_WPE
#else
#define WC_DUAL_WAVES_PER_EU 2
#define WC_WAVE2_WPE 1
#endif
#include "engine.hip"
