"""The Rust crate (rust/: the reference crate's public API over the C ABI)
cannot be compiled in this image (no cargo). Its raw bindings must still be a
faithful transcription of include/waffle_con.h: every function, with the same
parameter and return types, and every struct with the same fields in order
(a mismatch would be undefined behaviour at the FFI boundary). The public
modules must carry the reference's public API surface."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "waffle_con.h")
FFI = os.path.join(ROOT, "rust", "src", "ffi.rs")

_C_SCALARS = {"int": "c_int", "uint8_t": "u8", "uint32_t": "u32", "uint64_t": "u64", "int32_t": "i32",
              "int64_t": "i64", "double": "f64", "char": "c_char", "void": "()"}


def _strip_comments(s):
    s = re.sub(r"/\*.*?\*/", "", s, flags=re.S)
    return re.sub(r"//[^\n]*", "", s)


def _c_type(t):
    """C type text -> the canonical Rust spelling ('*const *const u8', 'u32', ...)."""
    t = t.replace("struct ", "").strip()
    # pointer levels from the right: "const uint8_t* const*" -> [const, const]
    parts = re.split(r"\*", t)
    base = parts[0].strip()
    quals = [p.strip() for p in parts[1:]]
    base_const = base.startswith("const ")
    base = base.replace("const ", "").strip()
    rust = _C_SCALARS.get(base, base)
    if not quals:
        return rust
    # innermost pointer's constness is the base's; outer ones follow the '*'s
    consts = [base_const] + [q == "const" for q in quals[:-1]]
    for c in consts:
        rust = ("*const " if c else "*mut ") + rust
    return rust


def _split_params(p):
    p = p.strip()
    if p in ("", "void"):
        return []
    return [x.strip() for x in p.split(",")]


def _c_param_type(p):
    m = re.match(r"(.*?)(\w+)$", p.strip(), re.S)
    return _c_type(m.group(1))


def header_functions():
    src = _strip_comments(open(HEADER).read())
    src = re.sub(r"#[^\n]*", "", src)
    out = {}
    for stmt in re.split(r"[;{}]", src):
        stmt = " ".join(stmt.split())
        m = re.match(r"^([A-Za-z_][\w \*]*?)\b(wc_\w+)\s*\((.*)\)$", stmt)
        if not m or m.group(1).startswith("typedef") or "extern" in m.group(1):
            continue
        out[m.group(2)] = (_c_type(m.group(1)), [_c_param_type(x) for x in _split_params(m.group(3))])
    return out


def header_structs():
    src = _strip_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"typedef struct (wc_\w+) \{(.*?)\} \1;", src, re.S):
        fields = []
        for decl in m.group(2).split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            mm = re.match(r"(.*?)(\w+)(\[\d+\])?$", decl)
            fields.append(mm.group(2))
        out[m.group(1)] = fields
    return out


def rust_functions():
    src = open(FFI).read()
    block = src[src.index('extern "C" {'):]
    out = {}
    for m in re.finditer(r"pub fn (wc_\w+)\((.*?)\)\s*(->\s*([^;]+))?;", block, re.S):
        params = [" ".join(x.split(":", 1)[1].split()) for x in _split_params(" ".join(m.group(2).split()))]
        ret = " ".join(m.group(4).split()) if m.group(4) else "()"
        out[m.group(1)] = (ret, params)
    return out


def rust_structs():
    src = open(FFI).read()
    out = {}
    for m in re.finditer(r"pub struct (wc_\w+) \{(.*?)\n\}", src, re.S):
        out[m.group(1)] = re.findall(r"pub (\w+):", m.group(2))
    return out


def test_every_header_function_is_bound_with_the_same_types():
    h, r = header_functions(), rust_functions()
    assert len(h) >= 40
    assert sorted(h) == sorted(r), (sorted(set(h) ^ set(r)))
    for name, (ret, params) in h.items():
        rret, rparams = r[name]
        assert rret == ret, (name, rret, ret)
        assert rparams == params, (name, rparams, params)


def test_every_header_struct_has_the_same_fields_in_order():
    h, r = header_structs(), rust_structs()
    assert {"wc_config", "wc_problem", "wc_chain_problem", "wc_dual_view", "wc_stats", "wc_dwfa_job",
            "wc_service_stats"} <= set(h)
    for name, fields in h.items():
        assert r.get(name) == fields, (name, r.get(name), fields)


def test_error_codes_match():
    hsrc = open(HEADER).read()
    rsrc = open(FFI).read()
    hc = dict(re.findall(r"(WC_(?:OK|E_\w+)) = (\d+)", hsrc))
    rc = dict(re.findall(r"pub const (WC_(?:OK|E_\w+)): c_int = (\d+);", rsrc))
    assert hc == rc


def test_public_api_surface_matches_the_reference():
    """The public items a user of waffle_con v0.4.4 calls."""
    want = {
        "cdwfa_config.rs": ["pub enum ConsensusCost", "L1Distance", "L2Distance", "pub struct CdwfaConfig",
                            "pub struct CdwfaConfigBuilder", "pub fn build(", "impl Default for CdwfaConfig"],
        "consensus.rs": ["pub struct Consensus ", "pub fn new(sequence: Vec<u8>, consensus_cost: ConsensusCost",
                         "pub fn sequence(&self) -> &[u8]", "pub fn scores(&self) -> &[usize]",
                         "pub struct ConsensusDWFA<'a>", "pub fn with_config(config: CdwfaConfig)",
                         "pub fn add_sequence(&mut self, sequence: &'a [u8])",
                         "pub fn add_sequence_offset(&mut self, sequence: &'a [u8], last_offset: Option<usize>)",
                         "pub fn consensus(&self) -> Result<Vec<Consensus>, Box<dyn std::error::Error>>",
                         "pub fn sequences(&self)", "pub fn consensus_cost(&self)", "pub fn alphabet(&self)"],
        "dual_consensus.rs": ["pub struct DualConsensus ", "pub fn is_dual(&self)", "pub fn consensus1(&self)",
                              "pub fn consensus2(&self) -> Option<&Consensus>", "pub fn is_consensus1(&self)",
                              "pub fn scores1(&self) -> &[Option<usize>]", "pub fn scores2(&self)",
                              "pub struct DualConsensusDWFA<'a>",
                              "pub fn consensus(&self) -> Result<Vec<DualConsensus>, Box<dyn std::error::Error>>"],
        "priority_consensus.rs": ["pub struct PriorityConsensus ", "pub fn consensuses(&self) -> &[Vec<Consensus>]",
                                  "pub fn sequence_indices(&self) -> &[usize]", "pub struct PriorityConsensusDWFA<'a>",
                                  "pub fn add_sequence_chain(&mut self, sequences: Vec<&'a [u8]>)",
                                  "pub fn add_seeded_sequence_chain(&mut self, sequences: Vec<&'a [u8]>, "
                                  "offsets: Vec<Option<usize>>,",
                                  "pub fn consensus(&self) -> Result<PriorityConsensus, Box<dyn std::error::Error>>",
                                  "Must provide a non-empty sequences Vec",
                                  "Expected sequences Vec of length {}, but got one of length {}"],
        "sequence_alignment.rs": ["pub fn wfa_ed(v1: &[u8], v2: &[u8]) -> usize",
                                  "pub fn wfa_ed_config(v1: &[u8], v2: &[u8], require_both_end: bool, "
                                  "wildcard: Option<u8>) -> usize"],
        "example_gen.rs": ["pub fn generate_test(alphabet_size: u8, seq_len: usize, num_samples: usize, "
                           "error_rate: f64) -> (Vec<u8>, Vec<Vec<u8>>)"],
        # dynamic_wfa.rs:12-265
        "dynamic_wfa.rs": ["#[derive(Clone, Debug, Eq, Hash, PartialEq)] pub struct DWFALite",
                           "impl Default for DWFALite",
                           "pub fn new(wildcard: Option<u8>, allow_early_termination: bool) -> DWFALite",
                           "pub fn set_offset(&mut self, offset: usize)",
                           "pub fn update(&mut self, baseline_seq: &[u8], other_seq: &[u8]) -> "
                           "Result<usize, Box<dyn std::error::Error>>",
                           "pub fn finalize(&mut self, baseline_seq: &[u8], other_seq: &[u8]) -> "
                           "Result<(), Box<dyn std::error::Error>>",
                           "pub fn maximum_baseline_distance(&self) -> usize",
                           "pub fn maximum_other_distance(&self) -> usize",
                           "pub fn reached_baseline_end(&self, baseline_seq: &[u8]) -> bool",
                           "pub fn get_extension_candidates(&self, baseline_seq: &[u8], other_seq: &[u8]) -> "
                           "HashMap<u8, usize>",
                           "use rustc_hash::FxHashMap as HashMap;",
                           "pub fn edit_distance(&self) -> usize", "pub fn wavefront(&self) -> &[usize]",
                           "Cannot push more bases after finalizing a DWFA", "Cannot finalize a DWFA twice.",
                           "ffi::wc_dwfa_batch"],
        # ragged or short inputs are refused before the ABI (never read past an array)
        "device.rs": ["expected {} offsets (one per read), got {}", "sequence chain {} has {} levels, expected {}",
                      "offsets of chain {} have {} entries, expected {}",
                      "expected {} seed groups (one per chain), got {}", ".collect::<Result<_, _>>()?"],
        # pqueue_tracker.rs:10-144
        "pqueue_tracker.rs": ["pub struct PQueueTracker",
                              "pub fn with_capacity(initial_size: usize, capacity_per_size: usize) -> PQueueTracker",
                              "pub fn insert(&mut self, value: usize)", "pub fn remove(&mut self, value: usize)",
                              "pub fn increment_threshold(&mut self)",
                              "pub fn increase_threshold(&mut self, new_threshold: usize)",
                              "pub fn process(&mut self, value: usize) -> Result<(), Box<dyn std::error::Error>>",
                              "pub fn processed(&self, value: usize) -> usize",
                              "pub fn at_capacity(&self, value: usize) -> bool", "pub fn len(&self) -> usize",
                              "pub fn unfiltered_len(&self) -> usize", "pub fn is_empty(&self) -> bool",
                              "pub fn threshold(&self) -> usize", "pub fn occupancy(&self, value: usize) -> usize",
                              "Capacity is full"],
        # multi_consensus.rs:11-65
        "multi_consensus.rs": ["#[derive(Debug, PartialEq)] pub struct MultiConsensus",
                               "pub fn new(consensuses: Vec<Consensus>, sequence_indices: Vec<usize>) -> "
                               "MultiConsensus",
                               "pub fn consensuses(&self) -> &[Consensus]",
                               "pub fn sequence_indices(&self) -> &[usize]"],
    }
    for f, items in want.items():
        src = " ".join(open(os.path.join(ROOT, "rust", "src", f)).read().split())
        for it in items:
            assert it in src, (f, it)
    # the reference's nine public modules (lib.rs:38-55), each a file of the crate
    lib_rs = open(os.path.join(ROOT, "rust", "src", "lib.rs")).read()
    for m in ("cdwfa_config", "consensus", "dual_consensus", "dynamic_wfa", "example_gen", "multi_consensus",
              "pqueue_tracker", "priority_consensus", "sequence_alignment"):
        assert "pub mod %s;" % m in lib_rs, m
        assert os.path.exists(os.path.join(ROOT, "rust", "src", m + ".rs")), m
    # the reference's FxHash types in the public signatures
    for f in ("consensus.rs", "dual_consensus.rs", "priority_consensus.rs"):
        assert "use rustc_hash::FxHashSet as HashSet;" in open(os.path.join(ROOT, "rust", "src", f)).read(), f
    cargo = open(os.path.join(ROOT, "rust", "Cargo.toml")).read()
    assert 'rustc-hash = "1.1.0"' in cargo
    assert 'name = "waffle_con"' in cargo and "build.rs" in cargo
    assert "gfx950" in open(os.path.join(ROOT, "rust", "build.rs")).read()
