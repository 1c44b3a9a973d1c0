//! MultiConsensus (multi_consensus.rs:11-65): the deprecated multi-consensus
//! result type, kept public by the reference. Consensuses are ordered by
//! sequence and the per-read assignment is renumbered to match.
use crate::consensus::Consensus;

/// multi_consensus.rs:11-16
#[derive(Debug, PartialEq)]
pub struct MultiConsensus {
    consensuses: Vec<Consensus>,
    sequence_indices: Vec<usize>,
}

impl MultiConsensus {
    /// multi_consensus.rs:25-55: a stable sort by sequence; read i's index
    /// follows its consensus to the new position
    pub fn new(consensuses: Vec<Consensus>, sequence_indices: Vec<usize>) -> MultiConsensus {
        let mut order: Vec<usize> = (0..consensuses.len()).collect();
        order.sort_by(|&i, &j| consensuses[i].sequence().cmp(consensuses[j].sequence()));
        let mut new_pos = vec![usize::MAX; consensuses.len()];
        for (pos, &old) in order.iter().enumerate() {
            new_pos[old] = pos;
        }
        let mut slots: Vec<Option<Consensus>> = consensuses.into_iter().map(Some).collect();
        let consensuses = order.iter().map(|&old| slots[old].take().unwrap()).collect();
        MultiConsensus { consensuses, sequence_indices: sequence_indices.iter().map(|&c| new_pos[c]).collect() }
    }

    /// multi_consensus.rs:58-60
    pub fn consensuses(&self) -> &[Consensus] {
        &self.consensuses
    }

    /// multi_consensus.rs:62-64
    pub fn sequence_indices(&self) -> &[usize] {
        &self.sequence_indices
    }
}
