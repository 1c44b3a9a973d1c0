// The dual engine with the linear-chain run-ahead call (namespace wcd): the
// launches of dual searches that ask for chains (WC_DUAL_CHAIN=<k>). The
// default builds leave the call out: the chains do not pay on this path's
// workloads and the call site costs the dual kernel registers.
// Same source as engine.hip, 256-thread workgroups.
#define WC_DUAL_CHAIN_CALL 1
#define WC_ENGINE_NS wcd
#include "engine.hip"
