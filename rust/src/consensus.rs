//! ConsensusDWFA (consensus.rs:76-365): the same constructors, accessors and
//! errors; consensus() runs the search on the MI355X (device::service_single).
use rustc_hash::FxHashSet as HashSet;

use crate::cdwfa_config::{CdwfaConfig, ConsensusCost};
use crate::device;

/// A final consensus result (consensus.rs:42-74)
#[derive(Clone, Debug, Default, PartialEq)]
pub struct Consensus {
    sequence: Vec<u8>,
    consensus_cost: ConsensusCost,
    scores: Vec<usize>,
}

impl Consensus {
    pub fn new(sequence: Vec<u8>, consensus_cost: ConsensusCost, scores: Vec<usize>) -> Consensus {
        Consensus { sequence, consensus_cost, scores }
    }

    pub fn sequence(&self) -> &[u8] {
        &self.sequence
    }

    pub fn consensus_cost(&self) -> ConsensusCost {
        self.consensus_cost
    }

    pub fn scores(&self) -> &[usize] {
        &self.scores
    }
}

/// consensus.rs:76-88
#[derive(Debug, Default)]
pub struct ConsensusDWFA<'a> {
    sequences: Vec<&'a [u8]>,
    offsets: Vec<Option<usize>>,
    config: CdwfaConfig,
    alphabet: HashSet<u8>,
}

impl<'a> ConsensusDWFA<'a> {
    /// consensus.rs:96
    pub fn with_config(config: CdwfaConfig) -> Result<ConsensusDWFA<'a>, Box<dyn std::error::Error>> {
        Ok(ConsensusDWFA { sequences: vec![], offsets: vec![], config, alphabet: Default::default() })
    }

    /// consensus.rs:110
    pub fn add_sequence(&mut self, sequence: &'a [u8]) -> Result<(), Box<dyn std::error::Error>> {
        self.add_sequence_offset(sequence, None)
    }

    /// consensus.rs:120
    pub fn add_sequence_offset(&mut self, sequence: &'a [u8], last_offset: Option<usize>) -> Result<(), Box<dyn std::error::Error>> {
        self.alphabet.extend(sequence.iter().cloned());
        if let Some(wc) = self.config.wildcard {
            self.alphabet.remove(&wc);
        }
        self.sequences.push(sequence);
        self.offsets.push(last_offset);
        Ok(())
    }

    /// consensus.rs:139-351, on the device. Re-entrant: any number of threads
    /// may call it at once (they share the device's submission service).
    pub fn consensus(&self) -> Result<Vec<Consensus>, Box<dyn std::error::Error>> {
        let prob = device::Problem::new(&self.sequences, &self.offsets)?;
        device::service_single(&self.config, &prob)
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
