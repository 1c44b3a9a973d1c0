// The 256-thread engines at 2 waves per SIMD (namespace wcl): a 256-VGPR
// budget, no register spills, 2 workgroups per CU. For launches that run few
// problems at once (one locus, a PriorityConsensusDWFA epoch with few live
// problems), where each workgroup's latency is all that matters and the chip
// has room to spare. Same source as engine.hip.
#define WC_LOWLAT 1
#define WC_ENGINE_NS wcl
#define WC_WAVES_PER_EU 2
#define WC_DUAL_WAVES_PER_EU 2
#include "engine.hip"
