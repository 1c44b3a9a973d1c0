"""MultiConsensus result type (multi_consensus.rs:10-65). A host-side container:
consensuses are sorted by sequence and sequence_indices re-mapped."""


class MultiConsensus:
    def __init__(self, consensuses, sequence_indices):
        order = sorted(range(len(consensuses)), key=lambda i: consensuses[i].sequence())
        reverse = [0] * len(consensuses)
        for new, old in enumerate(order):
            reverse[old] = new
        self._consensuses = [consensuses[i] for i in order]
        self._sequence_indices = [reverse[i] for i in sequence_indices]

    @classmethod
    def new(cls, consensuses, sequence_indices):
        return cls(consensuses, sequence_indices)

    def consensuses(self):
        return self._consensuses

    def sequence_indices(self):
        return self._sequence_indices

    def __eq__(self, other):
        return (isinstance(other, MultiConsensus) and self._consensuses == other._consensuses
                and self._sequence_indices == other._sequence_indices)
