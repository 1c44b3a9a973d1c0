"""GPU: the launch plans' workgroups per CU are what the hardware runs. gfx950
allocates a CU's 160 KB of LDS in granules of 1,280 bytes, more coarsely than
the runtime's occupancy query counts (tools/lds_occupancy.hip), so the
planner caps the query by the granule count of static + dynamic LDS
(engine.hip blocks_per_cu). The block dual build's 512-node pool fills 42
granules exactly at 3 workgroups per CU: 112 bytes more of static LDS (the
cooperative build's exchange, once in Ctl) ran cfg3 at 2 per CU, 3.18 ->
4.6 s, while the query still said 3. Results and counters must equal the
oracle's (dual_consensus.rs:240-787)."""
import pytest

import oracle_ffi as orc

pytestmark = pytest.mark.gpu

KEYS = ("updates", "w_out", "compares", "ed_increases", "finalizes", "pops", "nodes_explored", "nodes_ignored",
        "peak_queue_size", "row_bytes")


def test_dual_block_plan_three_per_cu(monkeypatch, capfd):
    """200-read dual problems on one CU (WC_DEVICE_SHARE on a fresh context),
    more of them than fit at once: the 4-wave block build at 3 per CU."""
    import waffle_con_amd as w
    from waffle_con_amd import _lib, synth
    from waffle_con_amd.cdwfa_config import CdwfaConfig
    for k in ("WC_WAVE", "WC_COOP", "WC_DUAL_LDS_KB", "WC_NARROW", "WC_LOWLAT", "WC_CU", "WC_GSTATE", "WC_DUAL_HOT",
              "WC_DUAL_CHAIN"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("WC_DEVICE_SHARE", "256")
    monkeypatch.setenv("WC_LAUNCH_LOG", "1")
    ctx = _lib.Context(0)
    probs = [synth.cfg3_locus(s, length=600) for s in range(4)]
    b = w.ResidentBatch(probs, context=ctx)
    _, st = b.dual_consensus(CdwfaConfig(), per_problem=True)
    log = capfd.readouterr().err
    launches = [ln for ln in log.splitlines() if "] launch sides=2" in ln]
    assert launches, log
    assert "per_cu=3 " in launches[0] and "wave=0" in launches[0] and "coop=0" in launches[0], launches[0]
    for p, pp in zip(probs, st["per_problem"]):
        _, ec = orc.dual_consensus(p, counters=True)
        for k in KEYS:
            assert pp[k] == ec[k], (k, pp[k], ec[k])
