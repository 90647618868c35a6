"""tools/shard_model.py's schedule replay (CPU): the per-rank projection of a logged sharded-proof schedule.

The library logs, per sharded proof, the order in which it starts exchanges, waits for them and runs compute between
(zk_prover_shard_schedule); simulate() replays that order for one rank on its own GPU.  These cases pin the replay
rules on hand-made schedules: a segment counts 1/G (all ranks serialised in the measurement) unless only the lead
rank ran it, exchanges queue FIFO on the exchange stream from their start, and a wait holds the compute stream only
until that exchange is done.
"""
import sys
from pathlib import Path

import pytest

sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "tools"))
import shard_model as sm  # noqa: E402


def sched(*entries):
    return {"world": 0, "measure": True, "entries": list(entries)}


def seg(ms, lead=False):
    return {"seg_ms": ms, "lead": lead}


def test_exchange_hidden_under_compute():
    G = 8
    b = 0.4 * (G - 1) * sm.LINK_BPS / 1e3  # 0.4 ms of link time + latency
    x = sm.xchg_ms(b, G)
    s = sched(seg(8.0), {"start": 0, "name": "a", "op": "ag", "bytes": b}, seg(16.0), {"wait": 0, "exposed_ms": 0})
    t, comp, xt, exposed, lead = sm.simulate(s, G)
    assert comp == pytest.approx(3.0) and t == pytest.approx(3.0) and exposed == 0 and xt == pytest.approx(x)
    tn = sm.simulate(s, G, overlap=False)[0]
    assert tn == pytest.approx(3.0 + x)


def test_exposed_when_compute_runs_out():
    G = 2
    b = 5.0 * sm.LINK_BPS / 1e3  # 5 ms on one link
    x = sm.xchg_ms(b, G)
    s = sched(seg(2.0), {"start": 0, "name": "a", "op": "a2a", "bytes": b}, seg(2.0), {"wait": 0, "exposed_ms": 0},
              seg(2.0))
    t, comp, _, exposed, _ = sm.simulate(s, G)
    assert comp == pytest.approx(3.0)
    assert t == pytest.approx(1.0 + x + 1.0) and exposed == pytest.approx(x - 1.0)


def test_fifo_exchange_stream_and_lead_segments():
    G = 4
    b = 1.0 * (G - 1) * sm.LINK_BPS / 1e3
    x = sm.xchg_ms(b, G)
    s = sched({"start": 0, "name": "a", "op": "ag", "bytes": b}, {"start": 1, "name": "b", "op": "ag", "bytes": b},
              seg(0.4), {"wait": 1, "exposed_ms": 0}, seg(0.5, lead=True))
    t, comp, _, exposed, lead = sm.simulate(s, G)
    # the second exchange starts when the first is done (one exchange stream per rank)
    assert t == pytest.approx(2 * x + 0.5) and lead == pytest.approx(0.5) and comp == pytest.approx(0.6)


def test_project_fits_replicated_and_divided_work():
    # serialised compute of G ranks = G R + S with R = 1, S = 16
    scheds = {G: {"device": sched(seg(1.0 * G + 16.0))} for G in (2, 4, 8)}
    pr = sm.project(scheds)["device"]
    assert pr["fit_all_rank_segments"]["replicated_ms_R"] == pytest.approx(1.0, abs=1e-3)
    assert pr["fit_all_rank_segments"]["divided_ms_S"] == pytest.approx(16.0, abs=1e-3)
    assert pr[8]["per_rank_ms"] == pytest.approx(1.0 + 2.0, abs=0.01)


def test_committed_projection_replays_from_its_schedules():
    """The projection committed with the round's final sharded schedules (bench.py's `model`) is
    what tools/shard_model.py computes from those schedules: the per-rank figures are reproducible from the file."""
    import json
    path = Path(__file__).resolve().parent.parent / "profiles" / "r06fin_shard_schedule_2p22.json"
    d = json.loads(path.read_text())
    pr = sm.project(d["schedules"])
    for kind, rec in d["projection"].items():
        for G in ("2", "4", "8"):
            assert pr[kind][int(G)]["per_rank_ms"] == pytest.approx(rec[G]["per_rank_ms"], abs=0.011), (kind, G)
            assert pr[kind][int(G)]["exposed_exchange_ms"] == pytest.approx(rec[G]["exposed_exchange_ms"], abs=0.011)
