"""Speculative batches and host-queued gossips (api.hip swim_step, dev_util.h tick_reset).

While no gossip slot is in use, one swim_step call is queued as SYNC-diff / member-kernel pairs with no host wait, and the
member kernel after which the gossip plane is needed raises the batch halt. User gossips (Cluster.spreadGossip,
ClusterImpl.java:208-211) are created by k_ug_create at P0 of the call's first tick, before that tick's member kernel,
so no member takes a slot in that tick: the speculative launch itself must see the slots already in use and halt the
batch there, or the gossips are never sent (GossipProtocolImpl.java:139-157). Only the randomized fuzz suite caught that
case once; these tests pin it deterministically: user gossips alone (no incarnation bump, no loss, so no member takes a
slot of its own) queued into an idle steady state at several tick offsets within the FD period, compared with the
oracle after every chunk, and every member but the origin must emit the GOSSIP event."""
import pytest

from swimhip import SimConfig

from parity_util import pair, run_lockstep

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("offset", [0, 1, 4, 9, 13])
def test_user_gossip_into_speculative_batch(oracle, engine, offset):
    n = 80
    cfg = SimConfig(n_members=n, record_events=True)
    o, e = pair(oracle, engine, cfg)
    # PRECONVERGED, no loss: no gossip is ever created by the protocol itself, so every swim_step call below starts
    # with the gossip plane idle and is queued as one speculative batch
    if offset:
        run_lockstep(o, e, offset, offset, f"idle to tick {offset}")
    origins = [7, 7, 41] if offset % 2 else [23]
    for c in (o, e):
        for i, m in enumerate(origins):
            c.spread_gossip(m, 0x5000 + 16 * offset + i)
    # the batch covers many ticks: a missing halt would run all of them without the gossip plane
    ev = run_lockstep(o, e, 60, 30, f"user gossips queued at tick {offset}")
    assert e.counters()["gossip_messages"] > 0
    seen = {}
    for x in ev:
        if x.isGossip():
            seen.setdefault(x.payload(), set()).add(x.observer)
    for i, m in enumerate(origins):
        assert seen.get(0x5000 + 16 * offset + i) == set(range(n)) - {m}, f"gossip {i} of member {m}"
    o.close()
    e.close()


def test_user_gossips_in_consecutive_batches(oracle, engine):
    """A user gossip queued while another one is still alive (no speculation then), then again after every slot has
    been recycled (speculation resumes): the two regimes back to back."""
    cfg = SimConfig(n_members=48, record_events=True)
    o, e = pair(oracle, engine, cfg)
    run_lockstep(o, e, 3, 3, "idle")
    for c in (o, e):
        c.spread_gossip(5, 1)
    run_lockstep(o, e, 40, 20, "first gossip")
    for c in (o, e):
        c.spread_gossip(9, 2)  # the first one is still held: the gossip plane is active
    run_lockstep(o, e, 600, 100, "second gossip, then both swept")
    for c in (o, e):
        c.spread_gossip(30, 3)  # idle again: queued into a speculative batch
    ev = run_lockstep(o, e, 80, 40, "third gossip")
    got = {x.observer for x in ev if x.isGossip() and x.payload() == 3}
    assert got == set(range(48)) - {30}
    o.close()
    e.close()
