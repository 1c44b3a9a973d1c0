"""CdwfaConfig / CdwfaConfigBuilder / ConsensusCost (cdwfa_config.rs:17-103)."""
import dataclasses
import enum
from typing import Optional


class ConsensusCost(enum.Enum):
    """cdwfa_config.rs:17-24."""
    L1Distance = 0
    L2Distance = 1


@dataclasses.dataclass
class CdwfaConfig:
    """cdwfa_config.rs:38-69; defaults from :71-103."""
    consensus_cost: ConsensusCost = ConsensusCost.L1Distance
    max_queue_size: int = 20
    max_capacity_per_size: int = 20
    max_return_size: int = 10
    max_nodes_wo_constraint: int = 1000
    min_count: int = 3
    min_af: float = 0.0
    weighted_by_ed: bool = False
    wildcard: Optional[int] = None
    dual_max_ed_delta: int = 20
    allow_early_termination: bool = False
    auto_shift_offsets: bool = True
    offset_window: int = 50
    offset_compare_length: int = 50

    def clone(self):
        return dataclasses.replace(self)


class CdwfaConfigBuilder:
    """derive_builder-style builder (`#[builder(default)]`, cdwfa_config.rs:38-39)."""

    def __init__(self):
        self._fields = {}

    def __getattr__(self, name):
        if name.startswith("_") or name not in CdwfaConfig.__dataclass_fields__:
            raise AttributeError(name)

        def setter(value):
            if name == "wildcard" and isinstance(value, (bytes, str)):
                value = ord(value)
            self._fields[name] = value
            return self

        return setter

    def build(self):
        return CdwfaConfig(**self._fields)
