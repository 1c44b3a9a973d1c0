// The consensus engines with their per-problem search state (heap, slot
// metadata, per-read nominations, work lists) in a per-workgroup HBM region
// instead of LDS: the path for problems whose state exceeds one workgroup's
// 160 KiB of LDS (thousands of reads, or queues of thousands of nodes), so
// the device accepts any number of reads, as the reference does
// (consensus.rs:110-134). Same source as engine.hip, namespace wcg.
#define WC_GLOBAL_STATE 1
#define WC_ENGINE_NS wcg
// register budget of the dual engine in this build (default: WC_WAVES_PER_EU)
#ifdef WC_GSTATE_DUAL_WPE
#define WC_DUAL_WAVES_PER_EU WC_GSTATE_DUAL_WPE
#endif
#include "engine.hip"
