"""SYNC_ACK resolution (k_ack_resolve): an answer sent in the tick its SYNC was merged is settled
from the write logs of its two ends instead of streamed. Bit-exact against the CPU oracle while the logs fill, overflow
and are bypassed (loss, kills, incarnation updates, metadata updates, graceful leaves, delays switched on mid-run,
several payloads to one receiver), and identical to the same run with every payload streamed (SWIM_NO_ACKRES)."""
import dataclasses
import os

import numpy as np
import pytest

from swimhip import ClusterConfig, SimConfig, SimulatedCluster

from parity_util import run_lockstep

pytestmark = pytest.mark.gpu

# SYNC every 10 ticks: many SYNC / SYNC_ACK pairs per tick, and receivers with several payloads
FAST_SYNC = ClusterConfig(syncInterval=1000)


def faults(c, phase):
    if phase == 0:
        c.set_default_loss(10)
    elif phase == 1:
        for m in (5, 77):
            c.kill(m)
        for m in range(20, 60, 3):
            c.update_incarnation(m)
        c.update_metadata(11)
    elif phase == 2:
        c.leave(90)
        c.set_default_link_settings(5, 150)  # delays from now on: late SYNCs and SYNC_ACKs are streamed


@pytest.mark.tape
def test_ack_resolution_parity_under_faults(oracle, engine):
    cfg = SimConfig(n_members=160, cluster=FAST_SYNC, delay_cap_ms=400, gossip_slot_cap=1 << 16)
    o, e = SimulatedCluster(oracle, cfg), SimulatedCluster(engine, dataclasses.replace(cfg, profile_all=True))
    for phase in range(3):
        for c in (o, e):
            faults(c, phase)
        run_lockstep(o, e, 120, 30, f"phase {phase}", events=False)
    assert o.events() == e.events()
    c = e.counters()
    assert c["ack_resolved_total"] > 0 and c["diff_msgs"] > 0
    assert c["ack_resolved"] == c["ack_resolved_total"]  # every tick timed
    e.close()
    o.close()


def test_ack_resolution_equals_streaming(engine):
    cfg = SimConfig(n_members=400, cluster=FAST_SYNC, gossip_slot_cap=1 << 16)
    runs = []
    for off in (False, True):
        if off:
            os.environ["SWIM_NO_ACKRES"] = "1"
        try:
            c = SimulatedCluster(engine, cfg)
        finally:
            os.environ.pop("SWIM_NO_ACKRES", None)
        hs = []
        for phase in range(2):
            faults(c, phase)
            c.step(90)
            hs.append(c.state_hash())
        runs.append((hs, c.events(), c.counters()))
        c.close()
    (ha, ea, ca), (hb, eb, cb) = runs
    for x, y in zip(ha, hb):
        assert np.array_equal(x, y)
    assert ea == eb
    assert ca["ack_resolved_total"] > 0 and cb["ack_resolved_total"] == 0
    for k in ("record_compares", "row_writes", "messages", "events", "sync_merges", "messages_lost"):
        assert ca[k] == cb[k], k


@pytest.mark.tape
@pytest.mark.parametrize("world", [2, 3])
def test_ack_resolution_sharded_parity(oracle, engine, world):
    """Row-sharded handles resolve SYNC_ACKs too: the responder's write-log prefix travels with the SYNC_ACK in exchange
    A. Bit-exact against the oracle under loss, kills, incarnation and metadata updates and a leave."""
    from swimhip.shard import ThreadShardGroup
    cfg = SimConfig(n_members=160, cluster=FAST_SYNC, gossip_slot_cap=1 << 16)
    o, e = SimulatedCluster(oracle, cfg), ThreadShardGroup(engine, cfg, world)
    for phase in range(2):
        for c in (o, e):
            faults(c, phase)
        run_lockstep(o, e, 120, 30, f"W={world} phase {phase}", events=False)
    for c in (o, e):
        c.leave(90)
    run_lockstep(o, e, 120, 30, f"W={world} leave", events=False)
    assert o.events() == e.events()
    assert e.counters()["ack_resolved_total"] > 0
    e.close()
    o.close()


@pytest.mark.parametrize("world", [1, 2, 4])
def test_ack_resolution_sharded_steady_accounting(engine, world):
    """C3-shaped steady state on W shards: the SYNC_ACKs are resolved (all but those whose receiver got several
    payloads in one tick), so the shards' k_sync_diff launches stream little more than the SYNC payloads, and the state
    equals the single-GPU run's."""
    from swimhip.shard import ThreadShardGroup
    cfg = SimConfig(n_members=3000, cluster=FAST_SYNC)
    c = SimulatedCluster(engine, cfg) if world == 1 else ThreadShardGroup(engine, cfg, world)
    c.run_periods(2)
    base = c.counters()
    c.run_periods(4)
    ctr = c.counters()
    d = {k: ctr[k] - base[k] for k in ("sync_merges", "ack_resolved_total", "diff_msgs_total")}
    assert d["sync_merges"] > 0 and d["ack_resolved_total"] * 4 > d["sync_merges"], d
    assert d["ack_resolved_total"] + d["diff_msgs_total"] == d["sync_merges"], d
    h = c.state_hash()
    c.close()
    if world > 1:
        ref = SimulatedCluster(engine, cfg)
        ref.run_periods(6)
        assert np.array_equal(ref.state_hash(), h)
        ref.close()


def test_diff_modes_agree(engine):
    """The SYNC diff's three ways of reading payloads give the same run: the 8-bit shadow plane (narrow list) with wide
    payloads in their own list (default), every payload on 4-B keys through the wide list (SWIM_NO_K8), and every
    payload streamed from the message buffer without SYNC_ACK resolution (SWIM_NO_ACKRES). Some members start at
    incarnation 60 and are bumped past the 8-bit escape while SYNCs run every tick, under loss, kills and a leave."""
    from swimhip import _abi
    cfg = SimConfig(n_members=400, cluster=FAST_SYNC, gossip_slot_cap=1 << 16)
    runs = []
    for env in (None, "SWIM_NO_K8", "SWIM_NO_ACKRES"):
        if env:
            os.environ[env] = "1"
        try:
            c = SimulatedCluster(engine, cfg)
        finally:
            if env:
                os.environ.pop(env, None)
        for m in (7, 31, 32, 200, 399):
            assert _abi.debug_set_incarnation(engine, c._h, m, 60) == 0
        hs = []
        for phase in range(3):
            faults(c, phase) if phase < 2 else c.leave(90)
            for m in (7, 32, 200):
                c.update_incarnation(m)
            c.step(60)
            hs.append(c.state_hash())
        runs.append((env, hs, c.events(), c.counters()))
        c.close()
    ref = runs[0]
    assert ref[3]["diff_msgs_total"] > 0
    for env, hs, ev, ctr in runs[1:]:
        for x, y in zip(ref[1], hs):
            assert np.array_equal(x, y), env
        assert ev == ref[2], env
        for k in ("record_compares", "row_writes", "messages", "events", "sync_merges", "messages_lost"):
            assert ctr[k] == ref[3][k], (env, k)
