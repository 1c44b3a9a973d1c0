//! PQueueTracker (pqueue_tracker.rs:10-144): counts of queued lengths above a
//! threshold, and a per-length cap on processed nodes. The search engines run
//! their own copy of this logic on the device (engine.hip TrackerRef); this is
//! the public host type, with the reference's methods, asserts and error.

/// pqueue_tracker.rs:10-21
#[derive(Debug)]
pub struct PQueueTracker {
    length_counts: Vec<usize>,
    total_count: usize,
    threshold: usize,
    processed_counts: Vec<usize>,
    capacity_per_size: usize,
}

impl PQueueTracker {
    /// pqueue_tracker.rs:28-36
    pub fn with_capacity(initial_size: usize, capacity_per_size: usize) -> PQueueTracker {
        PQueueTracker { length_counts: vec![0; initial_size], total_count: 0, threshold: 0,
                        processed_counts: vec![0; initial_size], capacity_per_size }
    }

    /// pqueue_tracker.rs:41-49
    pub fn insert(&mut self, value: usize) {
        if value >= self.length_counts.len() {
            self.length_counts.resize(value + 1, 0);
        }
        self.length_counts[value] += 1;
        if value >= self.threshold {
            self.total_count += 1;
        }
    }

    /// pqueue_tracker.rs:54-61
    pub fn remove(&mut self, value: usize) {
        assert!(self.length_counts[value] > 0);
        self.length_counts[value] -= 1;
        if value >= self.threshold {
            assert!(self.total_count > 0);
            self.total_count -= 1;
        }
    }

    /// pqueue_tracker.rs:64-66
    pub fn increment_threshold(&mut self) {
        self.increase_threshold(self.threshold + 1);
    }

    /// pqueue_tracker.rs:71-79: the counts of lengths in [old, new) leave the total
    pub fn increase_threshold(&mut self, new_threshold: usize) {
        assert!(new_threshold >= self.threshold);
        let old = self.threshold;
        for t in old..new_threshold {
            self.total_count -= self.length_counts[t];
        }
        self.threshold = new_threshold;
    }

    /// pqueue_tracker.rs:84-96
    pub fn process(&mut self, value: usize) -> Result<(), Box<dyn std::error::Error>> {
        if value >= self.processed_counts.len() {
            self.processed_counts.resize(value + 1, 0);
        }
        if self.processed_counts[value] >= self.capacity_per_size {
            return Err("Capacity is full".into());
        }
        self.processed_counts[value] += 1;
        Ok(())
    }

    /// pqueue_tracker.rs:101-107
    pub fn processed(&self, value: usize) -> usize {
        self.processed_counts.get(value).copied().unwrap_or(0)
    }

    /// pqueue_tracker.rs:112-114
    pub fn at_capacity(&self, value: usize) -> bool {
        self.processed(value) >= self.capacity_per_size
    }

    /// pqueue_tracker.rs:117-119
    pub fn len(&self) -> usize {
        self.total_count
    }

    /// pqueue_tracker.rs:122-124
    pub fn unfiltered_len(&self) -> usize {
        self.length_counts.iter().sum()
    }

    /// pqueue_tracker.rs:126-128
    pub fn is_empty(&self) -> bool {
        self.len() == 0
    }

    /// pqueue_tracker.rs:130-132
    pub fn threshold(&self) -> usize {
        self.threshold
    }

    /// pqueue_tracker.rs:137-143
    pub fn occupancy(&self, value: usize) -> usize {
        self.length_counts.get(value).copied().unwrap_or(0)
    }
}
