"""waffle_con on MI355X: the reference's consensus API (ConsensusDWFA,
DualConsensusDWFA, PriorityConsensusDWFA, CdwfaConfig) backed by a
device-resident HIP engine (waffle_con_amd/libwaffle_con.so, gfx950)."""
from ._lib import Context, WaffleConError, default_context
from .cdwfa_config import CdwfaConfig, CdwfaConfigBuilder, ConsensusCost
from .consensus import Consensus, ConsensusDWFA, consensus_batch
from .example_gen import generate_test

__all__ = [
    "CdwfaConfig", "CdwfaConfigBuilder", "ConsensusCost", "Consensus", "ConsensusDWFA", "consensus_batch",
    "generate_test", "Context", "WaffleConError", "default_context",
]
