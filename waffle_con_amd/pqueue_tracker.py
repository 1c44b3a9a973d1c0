"""PQueueTracker (pqueue_tracker.rs:10-144), the reference's public queue
bookkeeping type. The engines use a device copy of the same logic
(engine.hip TrackerRef); this host class keeps the public API."""
from ._lib import WaffleConError


class PQueueTracker:
    def __init__(self, initial_size, capacity_per_size):
        self._length_counts = [0] * initial_size
        self._total = 0
        self._threshold = 0
        self._processed = [0] * initial_size
        self._cap = capacity_per_size

    @classmethod
    def with_capacity(cls, initial_size, capacity_per_size):
        return cls(initial_size, capacity_per_size)

    def insert(self, value):
        if value >= len(self._length_counts):
            self._length_counts.extend([0] * (value + 1 - len(self._length_counts)))
        self._length_counts[value] += 1
        if value >= self._threshold:
            self._total += 1

    def remove(self, value):
        assert self._length_counts[value] > 0
        self._length_counts[value] -= 1
        if value >= self._threshold:
            assert self._total > 0
            self._total -= 1

    def increment_threshold(self):
        self.increase_threshold(self._threshold + 1)

    def increase_threshold(self, new_threshold):
        assert new_threshold >= self._threshold
        for t in range(self._threshold, new_threshold):
            self._total -= self._length_counts[t]
        self._threshold = new_threshold

    def process(self, value):
        if value >= len(self._processed):
            self._processed.extend([0] * (value + 1 - len(self._processed)))
        if self._processed[value] >= self._cap:
            raise WaffleConError("Capacity is full", 4)
        self._processed[value] += 1

    def processed(self, value):
        return 0 if value >= len(self._processed) else self._processed[value]

    def at_capacity(self, value):
        return self.processed(value) >= self._cap

    def len(self):
        return self._total

    def __len__(self):
        return self._total

    def unfiltered_len(self):
        return sum(self._length_counts)

    def is_empty(self):
        return self._total == 0

    def threshold(self):
        return self._threshold

    def occupancy(self, value):
        return 0 if value >= len(self._length_counts) else self._length_counts[value]
