//! DualConsensusDWFA (dual_consensus.rs:179-800): the same constructors,
//! accessors and errors; consensus() runs the search on the MI355X.
use rustc_hash::FxHashSet as HashSet;

use crate::cdwfa_config::{CdwfaConfig, ConsensusCost};
use crate::consensus::Consensus;
use crate::device;

/// dual_consensus.rs:52-177
#[derive(Debug, Clone)]
pub struct DualConsensus {
    consensus1: Consensus,
    consensus2: Option<Consensus>,
    is_consensus1: Vec<bool>,
    scores1: Vec<Option<usize>>,
    scores2: Vec<Option<usize>>,
}

/// dual_consensus.rs:66-75 (scores1/scores2 are not compared)
impl PartialEq for DualConsensus {
    fn eq(&self, other: &Self) -> bool {
        self.consensus1 == other.consensus1 && self.consensus2 == other.consensus2 && self.is_consensus1 == other.is_consensus1
    }
}

impl DualConsensus {
    /// dual_consensus.rs:79-99
    pub fn new(consensus1: Consensus, consensus2: Option<Consensus>, is_consensus1: Vec<bool>,
               scores1: Vec<Option<usize>>, scores2: Vec<Option<usize>>) -> Result<Self, Box<dyn std::error::Error>> {
        if is_consensus1.len() != scores1.len() || is_consensus1.len() != scores2.len() {
            return Err("is_consensus1, scores1, and scores2 must all be the same length".into());
        }
        Ok(Self { consensus1, consensus2, is_consensus1, scores1, scores2 })
    }

    pub fn is_dual(&self) -> bool {
        self.consensus2.is_some()
    }

    pub fn consensus1(&self) -> &Consensus {
        &self.consensus1
    }

    pub fn consensus2(&self) -> Option<&Consensus> {
        self.consensus2.as_ref()
    }

    pub fn is_consensus1(&self) -> &[bool] {
        &self.is_consensus1
    }

    pub fn scores1(&self) -> &[Option<usize>] {
        &self.scores1
    }

    pub fn scores2(&self) -> &[Option<usize>] {
        &self.scores2
    }
}

/// dual_consensus.rs:181-191
#[derive(Debug, Default)]
pub struct DualConsensusDWFA<'a> {
    sequences: Vec<&'a [u8]>,
    offsets: Vec<Option<usize>>,
    config: CdwfaConfig,
    alphabet: HashSet<u8>,
}

impl<'a> DualConsensusDWFA<'a> {
    /// dual_consensus.rs:199
    pub fn with_config(config: CdwfaConfig) -> Result<DualConsensusDWFA<'a>, Box<dyn std::error::Error>> {
        Ok(DualConsensusDWFA { sequences: vec![], offsets: vec![], config, alphabet: Default::default() })
    }

    /// dual_consensus.rs:211
    pub fn add_sequence(&mut self, sequence: &'a [u8]) -> Result<(), Box<dyn std::error::Error>> {
        self.add_sequence_offset(sequence, None)
    }

    /// dual_consensus.rs:221
    pub fn add_sequence_offset(&mut self, sequence: &'a [u8], last_offset: Option<usize>) -> Result<(), Box<dyn std::error::Error>> {
        self.alphabet.extend(sequence.iter().cloned());
        if let Some(wc) = self.config.wildcard {
            self.alphabet.remove(&wc);
        }
        self.sequences.push(sequence);
        self.offsets.push(last_offset);
        Ok(())
    }

    /// dual_consensus.rs:240-787, on the device (re-entrant)
    pub fn consensus(&self) -> Result<Vec<DualConsensus>, Box<dyn std::error::Error>> {
        let prob = device::Problem::new(&self.sequences, &self.offsets)?;
        device::service_dual(&self.config, &prob)
    }

    pub fn sequences(&self) -> &[&'a [u8]] {
        &self.sequences
    }

    pub fn consensus_cost(&self) -> ConsensusCost {
        self.config.consensus_cost
    }

    pub fn alphabet(&self) -> &HashSet<u8> {
        &self.alphabet
    }
}
