// The consensus engines with 128-thread workgroups (2 x wave64), namespace
// wcn: for problems of at most 128 reads. The single engine's linear-chain
// walk keeps one read per lane, so with 4 waves a 100-read locus fills 25 of
// 64 lanes per wave; every wave64 VALU instruction costs the SIMD 4 cycles
// whatever its active lanes, and at cfg2 the SIMDs are VALU-issue bound
// (SQ_ACTIVE_INST_VALU x 4 waves/SIMD ~ 70% of cycles, profiles/r02c_issue_view.json).
// Two waves carry the same reads at twice the lane occupancy: half the issue
// per locus, and the 2 waves/SIMD at 4 workgroups/CU leave 256 VGPRs per lane
// (no spills). Same source as engine.hip; LDS/HBM layouts are unchanged
// (sized for the 256-thread build).
#define WC_NARROW 1
#ifndef WC_NARROW_BLOCK
#define WC_NARROW_BLOCK 128
#endif
#define WC_BLOCK WC_NARROW_BLOCK  // (64: one-wave workgroups, an experiment build)
#define WC_ENGINE_NS wcn
#ifndef WC_NARROW_WAVES_PER_EU
#define WC_NARROW_WAVES_PER_EU 2
#endif
#define WC_WAVES_PER_EU WC_NARROW_WAVES_PER_EU
#include "engine.hip"
