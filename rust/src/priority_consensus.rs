//! PriorityConsensusDWFA (priority_consensus.rs:90-355): the same constructors,
//! accessors and errors; consensus() runs on the MI355X: this thread unwinds
//! the reference's LIFO work stack inside the library
//! (wc_service_priority_consensus) and every DualConsensusDWFA sub-problem runs
//! in the device's shared launches.
use rustc_hash::FxHashSet as HashSet;

use crate::cdwfa_config::{CdwfaConfig, ConsensusCost};
use crate::consensus::Consensus;
use crate::device;

/// priority_consensus.rs:64-88
#[derive(Clone, Debug, Default, PartialEq)]
pub struct PriorityConsensus {
    consensuses: Vec<Vec<Consensus>>,
    sequence_indices: Vec<usize>,
}

impl PriorityConsensus {
    pub fn new(consensuses: Vec<Vec<Consensus>>, sequence_indices: Vec<usize>) -> PriorityConsensus {
        PriorityConsensus { consensuses, sequence_indices }
    }

    pub fn consensuses(&self) -> &[Vec<Consensus>] {
        &self.consensuses
    }

    pub fn sequence_indices(&self) -> &[usize] {
        &self.sequence_indices
    }
}

/// priority_consensus.rs:94-106
#[derive(Debug, Default)]
pub struct PriorityConsensusDWFA<'a> {
    sequences: Vec<Vec<&'a [u8]>>,
    offsets: Vec<Vec<Option<usize>>>,
    seed_groups: Vec<Option<usize>>,
    config: CdwfaConfig,
    alphabet: HashSet<u8>,
}

impl<'a> PriorityConsensusDWFA<'a> {
    /// priority_consensus.rs:114
    pub fn with_config(config: CdwfaConfig) -> Result<PriorityConsensusDWFA<'a>, Box<dyn std::error::Error>> {
        Ok(PriorityConsensusDWFA { sequences: vec![], offsets: vec![], seed_groups: vec![], config,
                                   alphabet: Default::default() })
    }

    /// priority_consensus.rs:129
    pub fn add_sequence_chain(&mut self, sequences: Vec<&'a [u8]>) -> Result<(), Box<dyn std::error::Error>> {
        let offsets = vec![None; sequences.len()];
        self.add_seeded_sequence_chain(sequences, offsets, None)
    }

    /// priority_consensus.rs:141-167 (same errors and messages)
    pub fn add_seeded_sequence_chain(&mut self, sequences: Vec<&'a [u8]>, offsets: Vec<Option<usize>>,
                                     seed_group: Option<usize>) -> Result<(), Box<dyn std::error::Error>> {
        if sequences.is_empty() {
            return Err("Must provide a non-empty sequences Vec".into());
        }
        if !self.sequences.is_empty() && self.sequences[0].len() != sequences.len() {
            return Err(format!("Expected sequences Vec of length {}, but got one of length {}",
                               self.sequences[0].len(), sequences.len()).into());
        }
        for sequence in sequences.iter() {
            self.alphabet.extend(sequence.iter().cloned());
        }
        if let Some(wc) = self.config.wildcard {
            self.alphabet.remove(&wc);
        }
        self.sequences.push(sequences);
        self.offsets.push(offsets);
        self.seed_groups.push(seed_group);
        Ok(())
    }

    /// priority_consensus.rs:172-341, on the device (re-entrant)
    pub fn consensus(&self) -> Result<PriorityConsensus, Box<dyn std::error::Error>> {
        let prob = device::ChainProblem::new(&self.sequences, &self.offsets, &self.seed_groups)?;
        device::service_priority(&self.config, &prob)
    }

    pub fn sequences(&self) -> &[Vec<&'a [u8]>] {
        &self.sequences
    }

    pub fn consensus_cost(&self) -> ConsensusCost {
        self.config.consensus_cost
    }

    pub fn alphabet(&self) -> &HashSet<u8> {
        &self.alphabet
    }
}
