"""NetworkEmulator delays and counters on the CPU oracle (SEMANTICS.md §2): the GossipProtocolTest grid
(GossipProtocolTest.java:50-66,108-210: N members, loss %, mean delay ms) in the gossip-only harness (RUMOR mode, one
user gossip), and the emulator's sent / lost counters (NetworkEmulator.java:200-272)."""
import numpy as np
import pytest

from swimhip import ClusterConfig, SimConfig, _abi
from swimhip.cluster import SimulatedCluster

# GossipProtocolTest.experiments (:50-66): (members, loss %, mean delay ms)
GRID = [(2, 0, 2), (3, 0, 2), (5, 0, 2), (10, 0, 2), (10, 10, 2), (10, 25, 2), (10, 25, 100), (10, 50, 2),
        (50, 0, 2), (50, 10, 2), (50, 10, 100)]


def sweep_ticks(cfg: SimConfig):
    """ClusterMath.gossipTimeoutToSweep (ClusterMath.java:99-113) in ticks: 2 (spread + 1) gossip periods."""
    c = cfg.cluster
    spread = c.gossipRepeatMult * int(cfg.n_members).bit_length()
    return 2 * (spread + 1) * (c.gossipInterval // cfg.tick_ms)


def run_grid_case(lib, n, loss, delay, seed=0x5EED5EED):
    cfg = SimConfig(n_members=n, mode=_abi.MODE_RUMOR, record_events=True, seed=seed, emulator_counters=True,
                    delay_cap_ms=100)
    c = SimulatedCluster(lib, cfg)
    c.set_default_link_settings(loss, delay)
    c.spread_gossip(0, 0xC0FFEE)
    # awaitFullCompletion (:76-77): the whole gossip lifetime, plus the longest delay a send can get (22 ticks at 100 ms)
    c.step(sweep_ticks(cfg) + 30)
    return c


@pytest.mark.parametrize("n,loss,delay", GRID)
def test_gossip_protocol_grid(oracle, n, loss, delay):
    c = run_grid_case(oracle, n, loss, delay)
    got = [e.observer for e in c.events() if e.isGossip()]
    # every other member receives the gossip exactly once (:128-160: the latch and the double-delivery check)
    assert len(got) == len(set(got)), "double delivery"
    assert sorted(got) == list(range(1, n)) or loss >= 25, sorted(got)
    em = c.emulator_counters()
    sent, lost = int(em[:, 0].sum()), int(em[:, 1].sum())
    attempts = (sent + lost) // 2  # tryFail counts every send, tryDelay the ones that survived
    assert (sent + lost) % 2 == 0
    assert attempts == c.counters()["gossip_messages"]  # gossip only, nobody dead: every GOSSIP_REQ reached the emulator
    if loss == 0:
        assert lost == 0
    elif attempts >= 200:
        assert abs(lost / attempts - loss / 100) < 0.1, (lost, attempts)


def test_delay_shifts_dissemination(oracle):
    """The same gossip over 100 ms mean delays reaches the members later than over 2 ms ones (ticks of 100 ms: a
    2 ms mean never delays a message by a tick, a 100 ms mean does for ~37 % of them)."""
    def mean_tick(delay):
        c = run_grid_case(oracle, 50, 0, delay)
        ticks = [e.tick for e in c.events() if e.isGossip()]
        assert len(ticks) == 49
        return np.mean(ticks)
    assert mean_tick(100) > mean_tick(2) + 0.5


def test_link_settings_validation(oracle):
    c = SimulatedCluster(oracle, SimConfig(n_members=8))
    with pytest.raises(Exception):
        c.set_default_link_settings(0, 1200)  # past 11 x tick_ms: delays of 256 ticks would be reachable
    c.set_default_link_settings(5, 1100)
    c.set_link_settings(1, 2, 0, 300)
    c.step(20)


def test_counters_full_mode(oracle):
    """FD / SYNC / metadata messages count on the sender's emulator too: with no loss every send that reached the
    emulator counts twice; a dead destination refuses the connection before the emulator (not counted)."""
    cfg = SimConfig(n_members=16, cluster=ClusterConfig(syncInterval=2000), emulator_counters=True, delay_cap_ms=300)
    c = SimulatedCluster(oracle, cfg)
    c.set_default_link_settings(0, 300)
    c.step(60)
    em = c.emulator_counters()
    ctr = c.counters()
    assert int(em[:, 1].sum()) == 0
    assert int(em[:, 0].sum()) == 2 * (ctr["messages"] + ctr["gossip_messages"])
    c.kill(3)
    c.step(200)
    em2 = c.emulator_counters()
    ctr2 = c.counters()
    # sends to the dead member fail before the emulator: fewer emulator sends than messages attempted
    assert int(em2[:, 0].sum()) < 2 * (ctr2["messages"] + ctr2["gossip_messages"])
    assert int(em2[:, 1].sum()) == 0
