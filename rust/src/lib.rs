/*!
# waffle_con on AMD MI355X

The public API of `waffle_con` v0.4.4 (`cdwfa_config`, `consensus`,
`dual_consensus`, `dynamic_wfa`, `example_gen`, `multi_consensus`,
`pqueue_tracker`, `priority_consensus`, `sequence_alignment`)
with the dynamic-WFA consensus search running on an MI355X (gfx950): every
`consensus()` call goes to the device library built from
`../waffle_con_amd/csrc` (C ABI: `../include/waffle_con.h`, raw bindings in
[`ffi`]). Results, splits, scores and their order are bit-identical to the CPU
crate's. A caller switches the dependency and keeps its code:

```no_run
use waffle_con::consensus::ConsensusDWFA;

let sequences = [b"ACGT".to_vec(), b"ACCGT".to_vec(), b"ACCCGT".to_vec()];
let mut cdwfa: ConsensusDWFA = Default::default();
for s in sequences.iter() {
    cdwfa.add_sequence(s).unwrap();
}
let consensuses = cdwfa.consensus().unwrap();
assert_eq!(consensuses[0].sequence(), sequences[1]);
assert_eq!(consensuses[0].scores(), &[1, 0, 1]);
```

`consensus(&self)` is re-entrant, as in the reference: any number of host
threads may call it at once. The calls of a process share one submission
service per device (`wc_service_*`: persistent engine launches, one workgroup
per locus in flight). The device is `WAFFLE_CON_DEVICE` (default 0). Many loci
at once can also go through [`device::consensus_batch`] and friends (one
launch over the whole batch).

**Build status.** This crate has not been compiled or type-checked: the build
image has no `cargo`/`rustc` and no crate registry (`rustc-hash`,
`priority-queue` and `derive_builder` are crates.io dependencies). What is
checked, on the CPU, is the text: `tests/test_rust_crate.py` matches every
`ffi` declaration and `#[repr(C)]` struct against `include/waffle_con.h` and
the public surface against the reference's. The device paths these modules
call are parity-tested through the same C ABI from Python (`tests/test_gpu_*`,
e.g. `test_gpu_dwfa.py` for `DWFALite`'s update / finalize / candidates and
the insertion order its `get_extension_candidates` replays), but the Rust code
around those calls is not.
*/

/// Configuration for ConsensusDWFA (cdwfa_config.rs)
pub mod cdwfa_config;
/// ConsensusDWFA and Consensus (consensus.rs)
pub mod consensus;
/// Device access: the per-device service, batched calls, result decoding
pub mod device;
/// DualConsensusDWFA and DualConsensus (dual_consensus.rs)
pub mod dual_consensus;
/// DWFALite (dynamic_wfa.rs), its updates run on the device
pub mod dynamic_wfa;
/// generate_test (example_gen.rs), the reference's RNG restated in the library
pub mod example_gen;
/// Raw C ABI of the MI355X library (include/waffle_con.h)
pub mod ffi;
/// MultiConsensus (multi_consensus.rs), the deprecated result type
pub mod multi_consensus;
/// PQueueTracker (pqueue_tracker.rs)
pub mod pqueue_tracker;
/// PriorityConsensusDWFA and PriorityConsensus (priority_consensus.rs)
pub mod priority_consensus;
/// wfa_ed / wfa_ed_config (sequence_alignment.rs)
pub mod sequence_alignment;
