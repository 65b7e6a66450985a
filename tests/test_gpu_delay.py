"""Link delays (NetworkLinkSettings.evaluateDelay, SEMANTICS.md §2) and the emulator counters on the gfx950 engine,
against the CPU oracle tick by tick: the GossipProtocolTest grid (GossipProtocolTest.java:50-66), full-stack runs
where FD, SYNC, metadata and gossip messages all arrive late, the late PING_ACK that resolves the ping-req
subscriptions of its shared correlation id (FailureDetectorImpl.java:173,181-183), and metadata responses that
outlive their timeout. Bit-exact: state hashes, op counters, event streams and every member's emulator counters."""
import numpy as np
import pytest

from swimhip import ClusterConfig, SimConfig, _abi
from swimhip.cluster import SimulatedCluster

from parity_util import run_lockstep
from test_oracle_delay import GRID, sweep_ticks

pytestmark = pytest.mark.gpu


def both(oracle, engine, cfg):
    return SimulatedCluster(oracle, cfg), SimulatedCluster(engine, cfg)


def same_emulators(o, e, where):
    a, b = o.emulator_counters(), e.emulator_counters()
    bad = np.argwhere(a != b)
    assert len(bad) == 0, f"{where}: emulator counters differ at member {bad[0][0]}: {a[bad[0][0]]} vs {b[bad[0][0]]}"


@pytest.mark.parametrize("n,loss,delay", GRID)
def test_gossip_protocol_grid(oracle, engine, n, loss, delay):
    cfg = SimConfig(n_members=n, mode=_abi.MODE_RUMOR, record_events=True, emulator_counters=True, delay_cap_ms=100)
    o, e = both(oracle, engine, cfg)
    for c in (o, e):
        c.set_default_link_settings(loss, delay)
        c.spread_gossip(0, 0xC0FFEE)
        c.spread_gossip(n - 1, 0xBEEF)
    run_lockstep(o, e, sweep_ticks(cfg) + 30, 5, f"grid N={n} loss={loss} delay={delay}")
    same_emulators(o, e, "grid")


@pytest.mark.tape
@pytest.mark.parametrize("delay", [100, 400, 1100])
def test_full_stack_delays(oracle, engine, delay):
    """Every message kind late: pings and acks past the ping timeout (ping-req then resolves on the late direct ack),
    SYNC / SYNC_ACK payloads stored as sent, metadata responses past their timeout (1100 ms mean: ~6 % of them)."""
    # 1100 ms means: most FD rounds time out, so suspicion gossips pile up (more slots than the 64 per member default)
    cfg = SimConfig(n_members=40, cluster=ClusterConfig(syncInterval=3000, metadataTimeout=1000), record_events=True,
                    emulator_counters=True, delay_cap_ms=1100, gossip_slot_cap=8192)
    o, e = both(oracle, engine, cfg)
    for c in (o, e):
        c.set_default_link_settings(5, delay)
    run_lockstep(o, e, 200, 20, f"delay {delay} warm")
    for c in (o, e):
        c.kill(7)
        c.update_incarnation(3)
        c.update_metadata(11)
    run_lockstep(o, e, 400, 40, f"delay {delay} kill")
    same_emulators(o, e, f"delay {delay}")
    print(f"delay {delay}: {o.counters()['gossips_created']} gossips created, {o.counters()['messages']} messages")


def test_cold_join_with_delays(oracle, engine):
    cfg = SimConfig(n_members=48, cluster=ClusterConfig(seedMembers=[0, 5]), init_mode=_abi.INIT_COLD_JOIN,
                    record_events=True, emulator_counters=True, delay_cap_ms=300)
    o, e = both(oracle, engine, cfg)
    for c in (o, e):
        c.set_default_link_settings(0, 300)
    run_lockstep(o, e, 300, 25, "cold join, 300 ms delays")
    same_emulators(o, e, "cold join")


def test_late_direct_ack(oracle, engine):
    """B's acks to A are slow (mean 500 ms past a 500 ms ping timeout) and B cannot answer the helpers: A's direct
    timeout starts the ping-req round, and a direct PING_ACK that lands before its deadline resolves the helpers'
    subscriptions on the same correlation id (ALIVE, no suspicion); a later one finds none."""
    n = 6
    cfg = SimConfig(n_members=n, record_events=True, emulator_counters=True, delay_cap_ms=500)
    o, e = both(oracle, engine, cfg)
    a, b = 0, 1
    for c in (o, e):
        c.set_link_settings(b, a, 0, 500)
        for h in range(2, n):
            c.block(b, h)
    run_lockstep(o, e, 400, 20, "late direct ack")
    same_emulators(o, e, "late ack")


def test_per_link_delays_and_partition(oracle, engine):
    """Two custom mean delays on some links, the default on the rest; a partition overwrites the cross-group ones
    (block), unblock_all clears them; a loss-only setLinkSettings sets the link's delay to 0."""
    n = 32
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(syncInterval=2000), record_events=True, emulator_counters=True,
                    delay_cap_ms=800)
    o, e = both(oracle, engine, cfg)
    g = np.array([0] * (n // 2) + [1] * (n // 2), dtype=np.uint32)
    for c in (o, e):
        c.set_default_link_settings(2, 200)
        for s in range(0, n, 3):
            c.set_link_settings(s, (s + 5) % n, 10, 800)
            c.set_link_settings((s + 7) % n, s, 0, 50)
        c.set_link_loss(4, 9, 20)
    run_lockstep(o, e, 150, 25, "per-link delays")
    for c in (o, e):
        c.partition(g)
    run_lockstep(o, e, 250, 50, "partitioned")
    for c in (o, e):
        c.unblock_all()
        c.set_default_link_settings(0, 100)
    run_lockstep(o, e, 300, 50, "healed")
    same_emulators(o, e, "per-link")


def test_delay_cap_enforced(engine):
    c = SimulatedCluster(engine, SimConfig(n_members=8, delay_cap_ms=100))
    c.set_default_link_settings(0, 2)  # never reaches a tick: no cap needed
    with pytest.raises(Exception):
        c.set_default_link_settings(0, 300)  # above delay_cap_ms
    c.close()
    c = SimulatedCluster(engine, SimConfig(n_members=8))
    c.set_default_link_settings(0, 4)
    with pytest.raises(Exception):
        c.set_default_link_settings(0, 100)
    with pytest.raises(Exception):
        c.emulator_counters()  # SWIM_FLAG_EMULATOR_COUNTERS not set
    c.close()


# ---- the same on sharded handles: delayed SYNC / SYNC_ACK messages stored on the receiver's shard,
# delayed gossip receipts queued on the target's shard and replicated through exchange B, emulator counters summed


def sharded(oracle, engine, cfg, world):
    from swimhip.shard import ThreadShardGroup
    return SimulatedCluster(oracle, cfg), ThreadShardGroup(engine, cfg, world)


@pytest.mark.parametrize("n,loss,delay", [g for g in GRID if g[0] >= 10])
def test_gossip_protocol_grid_sharded(oracle, engine, n, loss, delay):
    """RUMOR mode on 2 slot shards: each shard's own gossips' sends, delays and counters."""
    cfg = SimConfig(n_members=n, mode=_abi.MODE_RUMOR, record_events=True, emulator_counters=True, delay_cap_ms=100)
    o, e = sharded(oracle, engine, cfg, 2)
    for c in (o, e):
        c.set_default_link_settings(loss, delay)
        c.spread_gossip(0, 0xC0FFEE)
        c.spread_gossip(n - 1, 0xBEEF)
    run_lockstep(o, e, sweep_ticks(cfg) + 30, 5, f"grid x2 N={n} loss={loss} delay={delay}")
    same_emulators(o, e, "grid x2")
    e.close()


@pytest.mark.tape
@pytest.mark.parametrize("delay,world", [(100, 2), (400, 3), (1100, 2)])
def test_full_stack_delays_sharded(oracle, engine, delay, world):
    """Row-sharded: every message kind late, kills, incarnation and metadata updates (the grid of the unsharded case)."""
    cfg = SimConfig(n_members=40, cluster=ClusterConfig(syncInterval=3000, metadataTimeout=1000), record_events=True,
                    emulator_counters=True, delay_cap_ms=1100, gossip_slot_cap=8192)
    o, e = sharded(oracle, engine, cfg, world)
    for c in (o, e):
        c.set_default_link_settings(5, delay)
    run_lockstep(o, e, 200, 20, f"x{world} delay {delay} warm")
    for c in (o, e):
        c.kill(7)
        c.update_incarnation(3)
        c.update_metadata(11)
    run_lockstep(o, e, 400, 40, f"x{world} delay {delay} kill")
    same_emulators(o, e, f"x{world} delay {delay}")
    e.close()


def test_per_link_delays_and_partition_sharded(oracle, engine):
    n = 32
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(syncInterval=2000), record_events=True, emulator_counters=True,
                    delay_cap_ms=800)
    o, e = sharded(oracle, engine, cfg, 2)
    g = np.array([0] * (n // 2) + [1] * (n // 2), dtype=np.uint32)
    for c in (o, e):
        c.set_default_link_settings(2, 200)
        for s in range(0, n, 3):
            c.set_link_settings(s, (s + 5) % n, 10, 800)
            c.set_link_settings((s + 7) % n, s, 0, 50)
        c.set_link_loss(4, 9, 20)
    run_lockstep(o, e, 150, 25, "x2 per-link delays")
    for c in (o, e):
        c.partition(g)
    run_lockstep(o, e, 250, 50, "x2 partitioned")
    for c in (o, e):
        c.unblock_all()
        c.set_default_link_settings(0, 100)
    run_lockstep(o, e, 300, 50, "x2 healed")
    same_emulators(o, e, "x2 per-link")
    e.close()


def test_cold_join_with_delays_sharded(oracle, engine):
    cfg = SimConfig(n_members=48, cluster=ClusterConfig(seedMembers=[0, 5]), init_mode=_abi.INIT_COLD_JOIN,
                    record_events=True, emulator_counters=True, delay_cap_ms=300)
    o, e = sharded(oracle, engine, cfg, 2)
    for c in (o, e):
        c.set_default_link_settings(0, 300)
    run_lockstep(o, e, 300, 25, "x2 cold join, 300 ms delays")
    same_emulators(o, e, "x2 cold join")
    e.close()
