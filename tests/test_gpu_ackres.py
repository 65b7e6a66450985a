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
