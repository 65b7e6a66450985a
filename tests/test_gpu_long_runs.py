"""Runs longer than the 13-bit tick window of the engine's 16-bit holder entries (engine.h S16_*, SCRUB, SLIFE): slots
are recycled many times over 10^4 ticks, so stale entries of earlier gossips must read as never held (s_get) until the
periodic scrub clears them. Bit-exact against the CPU oracle, which keeps full ticks (state hashes include every
member's event-sequence hash)."""
import pytest

from swimhip import ClusterConfig, SimConfig, _abi

from parity_util import pair, run_lockstep

pytestmark = pytest.mark.gpu


@pytest.mark.tape
def test_rumor_long_run_slot_reuse(oracle, engine):
    cfg = SimConfig(n_members=200, mode=_abi.MODE_RUMOR, churn_per_period=8, gossip_slot_cap=1024)
    o, e = pair(oracle, engine, cfg)
    for c in (o, e):
        c.set_default_loss(5)
    run_lockstep(o, e, 12_000, 2_000, "rumor, 12 000 ticks", events=False)
    assert o.counters()["gossips_created"] > 4 * 1024  # every slot reused several times
    e.close()
    o.close()


@pytest.mark.tape
def test_full_long_run_slot_reuse(oracle, engine):
    cfg = SimConfig(n_members=120, cluster=ClusterConfig(seedMembers=[0]), gossip_slot_cap=1024)
    o, e = pair(oracle, engine, cfg)
    for c in (o, e):
        c.set_default_loss(10)
    run_lockstep(o, e, 4_000, 1_000, "full, loss", events=False)
    for c in (o, e):
        c.kill(7)
        c.update_incarnation(3)
    run_lockstep(o, e, 6_000, 1_000, "full, kill + update", events=False)  # (per-member event hashes compared)
    e.close()
    o.close()


@pytest.mark.tape
def test_fine_tick_long_run(oracle, engine):
    """A 10 ms tick (gossip interval = 20 ticks, so a slot's lifetime is ~2 000 ticks of the 4 096 its 16-bit holder
    entries allow): slots recycled over 24 000 ticks, bit-exact."""
    cfg = SimConfig(n_members=150, mode=_abi.MODE_RUMOR, churn_per_period=6, gossip_slot_cap=1024, tick_ms=10)
    o, e = pair(oracle, engine, cfg)
    for c in (o, e):
        c.set_default_loss(5)
    run_lockstep(o, e, 24_000, 4_000, "rumor, 10 ms ticks", events=False)
    assert o.counters()["gossips_created"] > 1024  # every slot reused
    e.close()
    o.close()


def test_tick_window_refused_at_create(engine):
    """tick_ms = 1 with the default 200 ms gossip interval: a gossip would live ~20 000 ticks, past the holder entries'
    4 096-tick window, so swim_create refuses the config instead of failing mid-run with E_SLIFE."""
    from swimhip import SimulatedCluster
    with pytest.raises(Exception, match=f"rc={_abi.SWIM_EINVAL}"):
        SimulatedCluster(engine, SimConfig(n_members=100, tick_ms=1))
