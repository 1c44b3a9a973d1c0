"""waffle_con on MI355X: the reference's consensus API (ConsensusDWFA,
DualConsensusDWFA, PriorityConsensusDWFA, CdwfaConfig, DWFALite, ...) backed by
a device-resident HIP engine (waffle_con_amd/libwaffle_con.so, gfx950)."""
from ._lib import Context, WaffleConError, default_context
from .batch import ResidentBatch
from .cdwfa_config import CdwfaConfig, CdwfaConfigBuilder, ConsensusCost
from .consensus import Consensus, ConsensusDWFA, consensus_batch
from .dual_consensus import DualConsensus, DualConsensusDWFA, dual_consensus_batch
from .dynamic_wfa import DWFALite
from .example_gen import generate_test
from .multi_consensus import MultiConsensus
from .pqueue_tracker import PQueueTracker
from .priority_consensus import PriorityConsensus, PriorityConsensusDWFA, priority_consensus_batch
from .sequence_alignment import wfa_ed, wfa_ed_batch, wfa_ed_config

__all__ = [
    "CdwfaConfig", "CdwfaConfigBuilder", "ConsensusCost", "Consensus", "ConsensusDWFA", "consensus_batch",
    "DualConsensus", "DualConsensusDWFA", "dual_consensus_batch", "PriorityConsensus", "PriorityConsensusDWFA",
    "priority_consensus_batch", "MultiConsensus", "PQueueTracker", "DWFALite", "generate_test", "wfa_ed", "wfa_ed_batch",
    "wfa_ed_config", "Context", "WaffleConError", "default_context", "ResidentBatch",
]
