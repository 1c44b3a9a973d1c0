// The dual engine with 1024-thread workgroups (16 x wave64, namespace wcv),
// for launches of at most one problem per CU (a DualConsensusDWFA batch of a
// few loci; a PriorityConsensusDWFA call whose sub-problems are few, e.g. one
// deep locus): each pop's per-read work (the heavy lists, the children's
// builds, the votes) spreads over 16 waves instead of 4. Opt-in (WC_CU=1):
// measured slower on one deep locus (cfg4 24.6 vs 22.8 s). A separate unit from
// engine_cu.hip: compiled together, the two kernels' shared callees got one
// register allocation and the single kernel spilled twice as much.
#define WC_CU 1
#define WC_DUAL_ONLY 1
#define WC_ENGINE_NS wcv
#define WC_BLOCK 1024
#define WC_WAVES_PER_EU 4
#define WC_DUAL_WAVES_PER_EU 4
#include "engine.hip"
