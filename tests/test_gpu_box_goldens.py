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


def c4_side_status(c, n, observers):
    """For each observer: the share of the other side it holds SUSPECT, and of its own side ALIVE."""
    half = n // 2
    out = []
    for o in observers:
        st = (c.row(o) >> np.uint64(32)) & np.uint64(3)
        other, own = (st[half:], st[:half]) if o < half else (st[:half], st[half:])
        out.append(((other == 2).mean(), (own == 1).mean(), int((st == 0).sum())))
    return out
