"""GPU parity where the votes are hardest: many small, noisy problems, whose
reads end their wavefronts on several tips (splits of 3, 5, 6 or 7: the
votes counted in 840ths of a read, engine.hip wave_votes_core) and whose few
reads make exact vote ties likely (those fall back to the reference's f64
read-order fold). Every problem's result, and the batch's work counters,
must equal the oracle's (consensus.rs:283-321, dual_consensus.rs:515-734)."""
import pytest

import oracle_ffi as orc

pytestmark = pytest.mark.gpu

hip = pytest.importorskip("hip_runner")

KEYS = ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored",
        "nodes_ignored", "row_bytes")


def _problems(n, length, reads, err, seed0):
    import waffle_con_amd as w
    return [w.generate_test(4, length, reads, err, seed0 + i)[1] for i in range(n)]


def _sum_counters(outs):
    tot = {k: 0 for k in KEYS}
    for _, c in outs:
        for k in KEYS:
            tot[k] += c[k]
    return tot


@pytest.mark.parametrize("err,seed0", [(0.12, 100), (0.2, 500)])
def test_single_votes_noisy_batch(err, seed0):
    probs = _problems(400, 60, 7, err, seed0)
    exp = []
    for p in probs:
        try:
            exp.append(orc.consensus(p, counters=True, min_count=2))
        except orc.OracleError as e:
            exp.append((e, None))
    got, st = hip.consensus_batch(probs, counters=True, min_count=2)
    for i, ((e, _), g) in enumerate(zip(exp, got)):
        if isinstance(e, Exception):
            assert isinstance(g, Exception) and g.code == e.code, (i, e, g)
        else:
            assert g == e, i
    ok = [x for x in exp if not isinstance(x[0], Exception)]
    if len(ok) == len(exp):
        tot = _sum_counters(ok)
        for k in KEYS:
            assert st[k] == tot[k], (k, st[k], tot[k])


def _dual(r):
    def cons(c):
        return {"sequence": c.sequence(), "scores": list(c.scores())}
    return {"consensus1": cons(r.consensus1()),
            "consensus2": None if r.consensus2() is None else cons(r.consensus2()),
            "is_consensus1": list(r.is_consensus1()), "scores1": list(r.scores1()), "scores2": list(r.scores2())}


@pytest.mark.parametrize("err,seed0", [(0.1, 900), (0.18, 1300)])
def test_dual_votes_noisy_batch(err, seed0):
    import waffle_con_amd as w
    a = _problems(200, 60, 5, err, seed0)
    b = _problems(200, 60, 5, err, seed0 + 5000)
    probs = [[x for pair in zip(p, q) for x in pair] for p, q in zip(a, b)]
    exp = []
    for p in probs:
        try:
            exp.append(orc.dual_consensus(p, counters=True, min_count=2))
        except orc.OracleError as e:
            exp.append((e, None))
    res, st = w.dual_consensus_batch(probs, hip.make_config(min_count=2), return_errors=True)
    for i, ((e, _), g) in enumerate(zip(exp, res)):
        if isinstance(e, Exception):
            assert isinstance(g, Exception) and g.code == e.code, (i, e, g)
        else:
            assert [_dual(r) for r in g] == e, i
    ok = [x for x in exp if not isinstance(x[0], Exception)]
    if len(ok) == len(exp):
        tot = _sum_counters(ok)
        for k in KEYS:
            assert st[k] == tot[k], (k, st[k], tot[k])
