"""BASELINE.json configs at their configured sizes, against oracle fixtures recorded on the GPU box.

The CPU oracle needs more host RAM at these sizes than the build container has (C3: ~210 GB at 100 000 members; C2
past period 3: the explicit infectedFrom sets of the SYNC re-spread storm; C4: 50 000 members' tables and the SUSPECT
gossips). tools/record_golden_box.py ran it on the GPU box's host (16 worker threads) and wrote, per period, a digest of
every member's state hashes (table row, FD / gossip lists and cursors, held gossips with infection periods, event
sequence hash, scalars), the eight deterministic op counters and a digest of that period's MembershipEvents
(tests/golden/{c3_full,c2_long,c4_50k}.json; the recording logs are under profiles/). Here the engine replays the same
scenarios (tests/golden/scenarios.py BOX_SCENARIOS) and must reproduce every record bit for bit."""
import dataclasses
import json
import sys
from pathlib import Path

import numpy as np
import pytest

GOLDEN = Path(__file__).resolve().parent / "golden"
sys.path.insert(0, str(GOLDEN))

from scenarios import BOX_SCENARIOS, record  # noqa: E402

from swimhip.cluster import SimulatedCluster  # noqa: E402

pytestmark = pytest.mark.gpu

COUNTERS = ["record_compares", "row_writes", "messages", "gossip_messages", "events", "messages_lost",
            "gossips_created", "sync_merges"]


def load(name):
    f = GOLDEN / f"{name}.json"
    if not f.exists():
        pytest.fail(f"{f} is missing: record it on the GPU box (tools/record_golden_box.py {name})")
    return json.loads(f.read_text())


def replay(engine, name, **cfg_changes):
    """The engine on scenario `name` for the fixture's periods, compared period by period; returns the open cluster."""
    want = load(name)
    cfg, _ = BOX_SCENARIOS[name]()
    c = SimulatedCluster(engine, dataclasses.replace(cfg, **cfg_changes))
    got = record(c, name, limit=len(want["periods"]))
    assert len(got["periods"]) == len(want["periods"])
    for g, w in zip(got["periods"], want["periods"]):
        assert g["counters"] == w["counters"], (
            f"{name} period {w['period']}: counters {dict(zip(COUNTERS, g['counters']))} != "
            f"{dict(zip(COUNTERS, w['counters']))}")
        assert g == w, f"{name} period {w['period']}: {g} != {w}"
    return c, want


def test_c3_headline_size_golden(engine):
    """C3 at 100 000 members in the bench's own configuration (SWIM_FLAG_PROFILE: speculative batches, SYNC_ACK
    resolution, the 16-bit diff): the 25 steady periods the default bench line runs (warm-up 5 + 20 timed), then two
    periods each after one updateIncarnation (gossip, SYNC re-spread, UPDATED events, metadata fetches)."""
    c, want = replay(engine, "c3_full")
    ce = c.counters()
    c.close()
    # every merged payload was either streamed by k_sync_diff or resolved from write logs (k_ack_resolve)
    assert ce["ack_resolved_total"] > 0
    assert ce["ack_resolved_total"] + ce["diff_msgs_total"] == ce["sync_merges"], ce
    steady = dict(zip(COUNTERS, want["periods"][24]["counters"]))
    assert steady["row_writes"] == 0 and steady["events"] == 0 and steady["sync_merges"] > 0  # the timed steady state
    last = dict(zip(COUNTERS, want["periods"][-1]["counters"]))
    assert last["events"] > 0 and last["gossips_created"] > 0


@pytest.mark.parametrize("shards", [1, 2])
def test_c2_configured_size_golden(engine, shards):
    """C2 at 10 000 members with 5 % loss past c2_full's 3 periods (the SYNC re-spread storm the C2 bench line times),
    on one handle and on one handle row-sharded over two shards (n_gpus = 2; one GPU: both shards on it)."""
    c, want = replay(engine, "c2_long", n_gpus=shards)
    c.close()
    assert len(want["periods"]) > 3


def c4_sides(c, n):
    """Every observer's table against the two sides of the partition (A = [0, n/2), B = the rest): per observer, the
    members of its own side it holds ALIVE, of the other side SUSPECT, and of the other side absent (removed)."""
    half = n // 2
    out = np.zeros((n, 3), dtype=np.int64)
    for o in range(n):
        st = (c.row(o) >> np.uint64(32)) & np.uint64(3)
        own, other = (st[:half], st[half:]) if o < half else (st[half:], st[:half])
        out[o] = ((own == 1).sum(), (other == 2).sum(), (other == 0).sum())
    return out


def test_c4_configured_size_golden(engine):
    """C4 at its configured 50 000 members through the periods the oracle's memory held on the GPU box: the partition
    from period 0, the first ping and ping-req timeouts across it (SUSPECT records and their gossips)."""
    c, want = replay(engine, "c4_50k")
    sides = [c.row(o) for o in (0, 24_999, 25_000, 49_999)]
    c.close()
    last = dict(zip(COUNTERS, want["periods"][-1]["counters"]))
    assert last["gossips_created"] > 10_000 and last["events"] == 0, last  # the SUSPECT wave has started
    for o, row in zip((0, 24_999, 25_000, 49_999), sides):
        st = (row >> np.uint64(32)) & np.uint64(3)
        own = st[:25_000] if o < 25_000 else st[25_000:]
        assert (own == 1).all(), o  # no member suspects its own side


def test_c4_long_partition_no_recovery_2000(engine):
    """MembershipProtocolTest.testLongNetworkPartitionNoRecovery (MembershipProtocolTest.java:313-366) on the C4 shape
    at 2 000 members, engine only: two halves blocked both ways from period 0. After the SUSPECT wave every member
    trusts its own side and suspects the whole other side; after the suspicion timeout (5 x ceilLog2(2000) = 55
    periods, ClusterMath.suspicionTimeout) and the DEAD-gossip storm it trusts its own side and the other side is
    gone: N x N/2 REMOVED events, nobody suspected."""
    from swimhip import ClusterConfig, SimConfig
    n = 2000
    c = SimulatedCluster(engine, SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0]), record_events=True,
                                           event_cap=1 << 22, pending_fetch_cap=4096, list_slack=4096))
    c.partition([0] * (n // 2) + [1] * (n // 2))
    c.run_periods(30)
    s = c4_sides(c, n)
    assert (s[:, 0] == n // 2).all() and (s[:, 1] == n // 2).all(), s.min(axis=0)
    c.run_periods(50)  # period 80: every suspicion timer has fired
    s = c4_sides(c, n)
    ev = c.events()
    c.close()
    assert (s[:, 0] == n // 2).all() and (s[:, 1] == 0).all() and (s[:, 2] == n // 2).all(), s.min(axis=0)
    removed = [e for e in ev if e.isRemoved()]
    assert len(removed) == n * (n // 2) and len(ev) == len(removed)
    half = n // 2
    assert all((e.observer < half) != (e.member < half) for e in removed)  # only the other side is removed


def test_c4_suspect_wave_8000(engine):
    """The C4 partition phase at 8 000 members (16 % of the configured size), engine only, to period 64, the last
    period before the first suspicion timer (5 x ceilLog2(8000) = 65 periods) can fire: every member holds its own side
    ALIVE and the whole other side SUSPECT (testLongNetworkPartitionNoRecovery's middle assertion), no event yet."""
    from swimhip import ClusterConfig, SimConfig
    n = 8000
    c = SimulatedCluster(engine, SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0]), record_events=True,
                                           pending_fetch_cap=4096, list_slack=4096))
    c.partition([0] * (n // 2) + [1] * (n // 2))
    c.run_periods(64)
    s = c4_sides(c, n)
    ctr = c.counters()
    c.close()
    assert (s[:, 0] == n // 2).all() and (s[:, 1] == n // 2).all(), s.min(axis=0)
    assert ctr["events"] == 0 and ctr["gossips_created"] > 100_000, ctr
