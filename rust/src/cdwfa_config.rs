/*!
Configuration of the consensus DWFA search: the reference's `CdwfaConfig`
(cdwfa_config.rs:38-103), same fields, defaults and builder methods. The
reference derives the builder with derive_builder; it is written out here.
```
use waffle_con::cdwfa_config::{CdwfaConfig, CdwfaConfigBuilder, ConsensusCost};
let config: CdwfaConfig = CdwfaConfigBuilder::default()
    .consensus_cost(ConsensusCost::L2Distance)
    .wildcard(Some(b'N'))
    .build()
    .unwrap();
```
*/
use crate::ffi;

/// cdwfa_config.rs:18-24
#[derive(Clone, Copy, Debug, Default, PartialEq)]
pub enum ConsensusCost {
    /// Minimizes the total edit distance across all sequences
    #[default]
    L1Distance,
    /// Minimizes the square of the edit distance across all sequences
    L2Distance,
}

/// cdwfa_config.rs:38-69
#[derive(Clone, Debug)]
pub struct CdwfaConfig {
    pub consensus_cost: ConsensusCost,
    pub max_queue_size: usize,
    pub max_capacity_per_size: usize,
    pub max_return_size: usize,
    pub max_nodes_wo_constraint: u64,
    pub min_count: u64,
    pub min_af: f64,
    pub weighted_by_ed: bool,
    pub wildcard: Option<u8>,
    pub dual_max_ed_delta: usize,
    pub allow_early_termination: bool,
    pub auto_shift_offsets: bool,
    pub offset_window: usize,
    pub offset_compare_length: usize,
}

/// cdwfa_config.rs:71-103
impl Default for CdwfaConfig {
    fn default() -> Self {
        Self {
            consensus_cost: ConsensusCost::L1Distance,
            max_queue_size: 20,
            max_capacity_per_size: 20,
            max_return_size: 10,
            max_nodes_wo_constraint: 1000,
            min_count: 3,
            min_af: 0.0,
            weighted_by_ed: false,
            wildcard: None,
            dual_max_ed_delta: 20,
            allow_early_termination: false,
            auto_shift_offsets: true,
            offset_window: 50,
            offset_compare_length: 50,
        }
    }
}

impl CdwfaConfig {
    /// The C ABI form (include/waffle_con.h wc_config)
    pub fn to_wc(&self) -> ffi::wc_config {
        ffi::wc_config {
            consensus_cost: match self.consensus_cost {
                ConsensusCost::L1Distance => 0,
                ConsensusCost::L2Distance => 1,
            },
            wildcard: self.wildcard.map_or(-1, |w| w as i32),
            max_queue_size: self.max_queue_size as u64,
            max_capacity_per_size: self.max_capacity_per_size as u64,
            max_return_size: self.max_return_size as u64,
            max_nodes_wo_constraint: self.max_nodes_wo_constraint,
            min_count: self.min_count,
            min_af: self.min_af,
            dual_max_ed_delta: self.dual_max_ed_delta as u64,
            offset_window: self.offset_window as u64,
            offset_compare_length: self.offset_compare_length as u64,
            weighted_by_ed: self.weighted_by_ed as u8,
            allow_early_termination: self.allow_early_termination as u8,
            auto_shift_offsets: self.auto_shift_offsets as u8,
            _pad: [0; 5],
        }
    }
}

/// The builder derive_builder generates for the reference (`#[builder(default)]`:
/// every unset field keeps CdwfaConfig::default()'s value).
#[derive(Clone, Debug, Default)]
pub struct CdwfaConfigBuilder {
    cfg: Option<CdwfaConfig>,
}

/// The error type derive_builder's build() returns (never produced: every field has a default).
#[derive(Debug)]
pub struct CdwfaConfigBuilderError(String);

impl std::fmt::Display for CdwfaConfigBuilderError {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        f.write_str(&self.0)
    }
}

impl std::error::Error for CdwfaConfigBuilderError {}

macro_rules! builder_setters {
    ($($field:ident : $t:ty),* $(,)?) => {
        impl CdwfaConfigBuilder {
            $(
                pub fn $field(&mut self, value: $t) -> &mut Self {
                    self.cfg.get_or_insert_with(CdwfaConfig::default).$field = value;
                    self
                }
            )*
        }
    };
}

builder_setters!(
    consensus_cost: ConsensusCost,
    max_queue_size: usize,
    max_capacity_per_size: usize,
    max_return_size: usize,
    max_nodes_wo_constraint: u64,
    min_count: u64,
    min_af: f64,
    weighted_by_ed: bool,
    wildcard: Option<u8>,
    dual_max_ed_delta: usize,
    allow_early_termination: bool,
    auto_shift_offsets: bool,
    offset_window: usize,
    offset_compare_length: usize,
);

impl CdwfaConfigBuilder {
    pub fn build(&self) -> Result<CdwfaConfig, CdwfaConfigBuilderError> {
        Ok(self.cfg.clone().unwrap_or_default())
    }
}
