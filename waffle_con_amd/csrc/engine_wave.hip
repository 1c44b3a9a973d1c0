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
#ifndef WC_DUAL_WAVES_PER_EU
#define WC_DUAL_WAVES_PER_EU 2
#endif
#include "engine.hip"
