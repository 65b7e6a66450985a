"""Parity of the gfx950 engine (libswimhip.so) with the CPU oracle, tick by tick, through the C ABI.

Compared after every chunk of ticks: per-member hashes of the membership row (incarnation, status, metadata bit and
suspicion deadline), the FD and gossip lists with their cursors, the held gossips with their infection periods, the
per-member MembershipEvent sequence, and the scalar protocol counters. The deterministic op counters are compared too,
and at the end the full MembershipEvent streams must be equal. Bit-exact; no tolerance.
The scenarios restate the reference's behavioural tests on the deterministic harness.
"""
import numpy as np
import pytest

from swimhip import ClusterConfig, SimConfig, _abi
from swimhip.cluster import SimulatedCluster

from parity_util import assert_same, pair, run_lockstep

pytestmark = pytest.mark.gpu


def test_c1_cold_join_kill_one(oracle, engine):
    """C1: 64 members cold-join through seed 0, member 63 is killed at period 10 (BASELINE.json configs[0])."""
    cfg = SimConfig(n_members=64, cluster=ClusterConfig(seedMembers=[0]), init_mode=_abi.INIT_COLD_JOIN,
                    record_events=True)
    o, e = pair(oracle, engine, cfg)
    ev = run_lockstep(o, e, 100, 5, "C1 join")
    assert sum(x.isAdded() for x in ev) == 64 * 63
    o.kill(63)
    e.kill(63)
    ev = run_lockstep(o, e, 400, 10, "C1 after kill")
    removed = [x for x in ev if x.isRemoved() and x.member == 63]
    assert sorted(x.observer for x in removed) == list(range(63))


def test_preconverged_loss(oracle, engine):
    """C2-shaped at reduced N: preconverged full views, 5 % loss on every link (BASELINE.json configs[1])."""
    cfg = SimConfig(n_members=300, record_events=True)
    o, e = pair(oracle, engine, cfg)
    o.set_default_loss(5)
    e.set_default_loss(5)
    ev = run_lockstep(o, e, 200, 10, "loss5")
    assert any(x.isUpdated() for x in ev)  # refutations happened


def test_partition_and_heal(oracle, engine):
    """C4-shaped at reduced N: two groups blocked both ways, suspicion timeout removes the other side, heal, SYNC
    recovery through the cross-group seed (MembershipProtocolTest.testNetworkPartitionDueNoOutboundThenRemove...)."""
    n = 48
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0, n - 1]), record_events=True)
    o, e = pair(oracle, engine, cfg)
    groups = np.array([0] * (n // 2) + [1] * (n // 2), dtype=np.uint32)
    o.partition(groups)
    e.partition(groups)
    run_lockstep(o, e, 350, 25, "partitioned")
    o.unblock_all()
    e.unblock_all()
    run_lockstep(o, e, 650, 25, "healed")


def _sametick_counter(lib, cluster, i):
    import ctypes as C
    fn = lib.swimdbg_counter
    fn.restype, fn.argtypes = C.c_uint64, [C.c_void_p, C.c_uint32]
    return fn(cluster._h, i)


@pytest.mark.parametrize("shards", [1, 2])
def test_sync_same_tick_resurrection(oracle, engine, monkeypatch, shards):
    """Several SYNC / SYNC_ACK payloads reach one receiver in the same tick, and an earlier one changes a row that a
    later one holds as it stood at the start of the tick. syncMembership filters each payload against the LIVE table
    (MembershipProtocolImpl.java:456-467): leaver 0's own `DEAD inc+1` (kept in its table, :197-206) removes it at R,
    then a SYNC from M > 0 still holding `0 ALIVE inc` (equal to R's start-of-tick row) re-adds it, because an absent
    row accepts any ALIVE record (MembershipRecord.java:67-69), with an ADDED after the metadata fetch. Fast SYNC
    (every 2 ticks) on 8 members makes such ticks frequent; the oracle counts them (SWIMREF_DEBUG)."""
    monkeypatch.setenv("SWIMREF_DEBUG", "1")
    cc = ClusterConfig(seedMembers=[0], syncInterval=200, syncTimeout=100)
    cfg = SimConfig(n_members=8, cluster=cc, record_events=True)
    o = SimulatedCluster(oracle, cfg)
    if shards == 1:
        e = SimulatedCluster(engine, cfg)
    else:
        from swimhip.shard import ThreadShardGroup
        e = ThreadShardGroup(engine, cfg, shards)
    run_lockstep(o, e, 7, 7, "warm")
    for c in (o, e):
        c.leave(0)
    run_lockstep(o, e, 60, 1, "leave 0, fast SYNC")
    assert _sametick_counter(oracle, o, 1) > 0, "the scenario did not occur"
    for c in (o, e):
        c.set_default_loss(20)
        c.leave(5)
        c.kill(3)
    run_lockstep(o, e, 200, 5, "leave 5, kill 3, loss 20")
    e.close()


@pytest.mark.parametrize("shards,cold", [(1, False), (2, False), (1, True), (2, True)])
def test_member_configs(oracle, engine, shards, cold):
    """Members with their own ClusterConfig (swim_set_member_config): FD timings and ping-req counts per member
    (FailureDetectorTest.testTrustedDespiteDifferentPingTimings, :150-178; the member's suspicion timeout follows its
    own pingInterval, MembershipProtocolImpl.java:597-606) and two syncGroups whose SYNC data the other side ignores
    (checkSyncGroup, :431-437), under loss and with a crash; bit-exact with the oracle. `cold`: every member joins at
    tick 0 through the seeds (start0), so its first ping follows its own pingInterval."""
    n = 60
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0, 55], syncInterval=3000), record_events=True,
                    init_mode=_abi.INIT_COLD_JOIN if cold else _abi.INIT_PRECONVERGED)
    o = SimulatedCluster(oracle, cfg)
    if shards == 1:
        e = SimulatedCluster(engine, cfg)
    else:
        from swimhip.shard import ThreadShardGroup
        e = ThreadShardGroup(engine, cfg, shards)
    for c in (o, e):
        for m in range(0, 10):
            c.set_member_config(m, ClusterConfig(pingInterval=500, pingTimeout=200, pingReqMembers=1))
        for m in range(10, 20):
            c.set_member_config(m, ClusterConfig(pingInterval=2000, pingTimeout=1000, pingReqMembers=4))
        for m in range(50, 60):
            c.set_member_config(m, ClusterConfig(syncGroup="b"))
        c.set_default_loss(10)
    run_lockstep(o, e, 150, 25, "mixed configs, loss 10")
    for c in (o, e):
        c.kill(12)
        c.kill(52)
    run_lockstep(o, e, 450, 50, "kills")
    e.close()


def test_fd_bad_network_per_member_unblock(oracle, engine):
    """FailureDetectorTest.testSuspectedMemberWithBadNetworkGetsPartitioned (:181-237) in lockstep: member 0 blocks
    every outbound link, then unblocks its own links only (a.networkEmulator().unblockAll(), per-link here)."""
    cc = ClusterConfig(pingInterval=200, pingTimeout=100, pingReqMembers=2, metadataTimeout=100)
    cfg = SimConfig(n_members=4, cluster=cc, tick_ms=10, record_events=True)
    o, e = pair(oracle, engine, cfg)
    for c in (o, e):
        c.block(0, 0, 1, 2, 3)
    run_lockstep(o, e, 100, 10, "0 blocked")
    for c in (o, e):
        c.unblock(0, 0, 1, 2, 3)
    run_lockstep(o, e, 400, 25, "0 unblocked")
    assert sorted(e.trusted(0)) == [0, 1, 2, 3]


def test_preconverged_sync_large(oracle, engine):
    """C3-shaped at reduced N: no loss, steady state; exercises periodic SYNC / SYNC_ACK merges."""
    cfg = SimConfig(n_members=1500)
    o, e = pair(oracle, engine, cfg)
    run_lockstep(o, e, 320, 80, "sync", events=False)


def test_fast_config_partition_recovery(oracle, engine):
    """MembershipProtocolTest's fast config (tick 10 ms, ping 200/100, sync 500/100, metadata 100), cold join of 5
    with every member a seed, a three-way partition until removal, then healing."""
    n = 5
    cc = ClusterConfig(seedMembers=list(range(n)), syncInterval=500, syncTimeout=100, pingInterval=200,
                       pingTimeout=100, metadataTimeout=100)
    cfg = SimConfig(n_members=n, cluster=cc, init_mode=_abi.INIT_COLD_JOIN, tick_ms=10, record_events=True)
    o, e = pair(oracle, engine, cfg)
    run_lockstep(o, e, 300, 20, "joined")
    g = np.array([0, 1, 2, 0, 1], dtype=np.uint32)
    o.partition(g)
    e.partition(g)
    run_lockstep(o, e, 500, 25, "partitioned")
    o.unblock_all()
    e.unblock_all()
    run_lockstep(o, e, 300, 25, "healed")


@pytest.mark.parametrize("loss", [0, 25])
def test_gossip_dissemination_update_incarnation(oracle, engine, loss):
    """GossipProtocolTest shape: 50 members, one incarnation bump disseminated under loss."""
    cfg = SimConfig(n_members=50, record_events=True)
    o, e = pair(oracle, engine, cfg)
    for c in (o, e):
        c.set_default_loss(loss)
        c.step(5)
        c.update_incarnation(0)
    run_lockstep(o, e, 120, 4, f"dissemination loss {loss}")
    for c in (o, e):
        c.update_incarnation(7)
        c.update_incarnation(8)
    run_lockstep(o, e, 200, 20, f"second wave loss {loss}")


def test_kill_many_with_loss(oracle, engine):
    """Churn under loss: several crashed members, suspicion storms and DEAD gossips with 10 % loss."""
    cfg = SimConfig(n_members=120, record_events=True)
    o, e = pair(oracle, engine, cfg)
    for c in (o, e):
        c.set_default_loss(10)
    run_lockstep(o, e, 50, 25, "warm")
    for victim in (3, 50, 51, 119):
        o.kill(victim)
        e.kill(victim)
    run_lockstep(o, e, 500, 50, "after kills")


def test_asymmetric_blocks_and_link_loss(oracle, engine):
    """FailureDetectorTest block matrices (:118-341) inside the full stack: one-directional blocks, per-link loss
    over a default loss, a partition that overwrites custom settings, unblock of single links, unblockAll."""
    n = 40
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0, 39]), record_events=True)
    o, e = pair(oracle, engine, cfg)
    for c in (o, e):
        c.set_default_loss(5)
        c.block(0, 1, 2, 3)
        c.block(7, 30)
        c.set_link_loss(5, 6, 60)
        c.set_link_loss(9, 10, 0)
    run_lockstep(o, e, 120, 20, "asymmetric")
    g = np.array([0] * 20 + [1] * 20, dtype=np.uint32)
    for c in (o, e):
        c.partition(g)
        c.set_link_loss(3, 25, 0)  # a custom setting made after the partition punches through it
    run_lockstep(o, e, 200, 40, "partition + custom")
    for c in (o, e):
        c.unblock(0, 1, 2)
        c.unblock(3, 25)
    run_lockstep(o, e, 100, 25, "single unblocks")
    for c in (o, e):
        c.unblock_all()
    run_lockstep(o, e, 200, 50, "unblockAll")


def test_graceful_leaves(oracle, engine):
    """Cluster.shutdown() -> leaveCluster: own DEAD record spread as gossip, REMOVED everywhere, the leaver stops when
    its gossip is swept (ClusterImpl.java:297-313, MembershipProtocolImpl.java:197-206); under loss, one at a time
    and two at once, plus an incarnation bump and a leave requested in the same tick."""
    cfg = SimConfig(n_members=120, record_events=True)
    o, e = pair(oracle, engine, cfg)
    run_lockstep(o, e, 30, 10, "warm")
    for c in (o, e):
        c.leave(7)
    run_lockstep(o, e, 60, 20, "leave 7")
    for c in (o, e):
        c.set_default_loss(10)
        c.leave(8)
        c.leave(90)
        c.update_incarnation(91)
        c.leave(91)
    ev = run_lockstep(o, e, 400, 50, "leave 8, 90, 91 under loss")
    assert {x.member for x in ev if x.isRemoved()} >= {8, 90, 91}


def test_user_gossips(oracle, engine):
    """Cluster.spreadGossip / listenGossips (ClusterImpl.java:208-216): user gossips beside the membership gossips,
    two from one member in one tick, under loss, from a member that leaves meanwhile; GOSSIP events must match."""
    cfg = SimConfig(n_members=90, record_events=True)
    o, e = pair(oracle, engine, cfg)
    run_lockstep(o, e, 12, 4, "warm")
    for c in (o, e):
        c.set_default_loss(10)
        c.spread_gossip(3, 0xDEADBEEF00000001)
        c.spread_gossip(3, 2)
        c.spread_gossip(70, 3)
        c.update_incarnation(3)
    ev = run_lockstep(o, e, 80, 10, "three user gossips under loss")
    for c in (o, e):
        c.spread_gossip(9, 4)
        c.leave(9)
    ev += run_lockstep(o, e, 150, 25, "gossip then leave")
    got = {}
    for x in ev:
        if x.isGossip():
            got.setdefault(x.payload(), set()).add(x.observer)
    assert got[0xDEADBEEF00000001] == set(range(90)) - {3}


def test_user_gossips_sharded(oracle, engine):
    from swimhip.shard import ThreadShardGroup
    cfg = SimConfig(n_members=75, record_events=True)
    o, e = SimulatedCluster(oracle, cfg), ThreadShardGroup(engine, cfg, 3)
    run_lockstep(o, e, 8, 4, "warm W=3")
    for c in (o, e):
        c.set_default_loss(5)
        for m in (1, 30, 31, 60):  # origins on every shard
            c.spread_gossip(m, 1000 + m)
    run_lockstep(o, e, 100, 20, "user gossips W=3")
    e.close()


@pytest.mark.parametrize("loss", [0, 10])
def test_rumor_mode(oracle, engine, loss):
    """RUMOR mode (C5 shape, SEMANTICS.md §9): churn rumors every period, plus a user gossip and a crash."""
    cfg = SimConfig(n_members=300, mode=_abi.MODE_RUMOR, churn_per_period=3, record_events=True)
    o, e = pair(oracle, engine, cfg)
    for c in (o, e):
        c.set_default_loss(loss)
    run_lockstep(o, e, 120, 20, f"rumor loss {loss}")
    for c in (o, e):
        c.spread_gossip(17, 99)
        c.kill(40)
    run_lockstep(o, e, 150, 30, f"rumor + user gossip + kill, loss {loss}")


def test_rumor_mode_sharded(oracle, engine):
    from swimhip.shard import ThreadShardGroup
    cfg = SimConfig(n_members=240, mode=_abi.MODE_RUMOR, churn_per_period=4, record_events=True)
    o, e = SimulatedCluster(oracle, cfg), ThreadShardGroup(engine, cfg, 2)
    run_lockstep(o, e, 200, 40, "rumor W=2")
    e.close()


@pytest.mark.parametrize("world", [3, 4])
def test_rumor_mode_slot_sharded_faults(oracle, engine, world):
    """RUMOR mode shards the gossips, not the observers: every shard runs all members and keeps
    the gossips it owns; the members' gossip counts are all-reduced every tick. Loss, a user gossip and crashes;
    events merged across shards in P4's gossip-id order."""
    from swimhip.shard import ThreadShardGroup
    cfg = SimConfig(n_members=300, mode=_abi.MODE_RUMOR, churn_per_period=5, record_events=True)
    o, e = SimulatedCluster(oracle, cfg), ThreadShardGroup(engine, cfg, world)
    for c in (o, e):
        c.set_default_loss(10)
    run_lockstep(o, e, 120, 20, f"rumor slot shards W={world}")
    for c in (o, e):
        c.spread_gossip(17, 99)
        c.kill(40)
        c.kill(41)
    run_lockstep(o, e, 150, 30, f"rumor slot shards + user gossip + kills W={world}")
    for m in (3, 150, 299):
        assert o.gossips(m) == e.gossips(m)
    cs = [s.counters()["gossips_created"] for s in e.shards]
    assert all(c > 0 for c in cs) and sum(cs) == o.counters()["gossips_created"]  # every shard owns a share
    e.close()


def test_joins_and_restarts(oracle, engine):
    """ClusterImpl.join0 of late processes (MembershipProtocolTest.testLimitedSeedMembers / testRestartFailedMembers
    shapes): dormant members join with their own seeds, crashed members are replaced by new ids, under 10 % loss."""
    cfg = SimConfig(n_members=60, cluster=ClusterConfig(seedMembers=[0]), init_mode=_abi.INIT_COLD_JOIN,
                    record_events=True, n_dormant=12)
    o, e = pair(oracle, engine, cfg)
    run_lockstep(o, e, 40, 10, "initial 48")
    for c in (o, e):
        c.join(48, [0])
        c.join(49, [5, 6])
        c.join(50, [])
    run_lockstep(o, e, 60, 15, "three joins")
    for c in (o, e):
        c.set_default_loss(10)
        c.kill(3)
        c.kill(4)
        c.join(51, [0, 1])
    run_lockstep(o, e, 250, 50, "kills + restart under loss")
    for c in (o, e):
        for m in range(52, 60):
            c.join(m, [m - 52, 48])
    run_lockstep(o, e, 200, 50, "eight joins at once")


def test_joins_sharded(oracle, engine):
    from swimhip.shard import ThreadShardGroup
    cfg = SimConfig(n_members=45, cluster=ClusterConfig(seedMembers=[0]), init_mode=_abi.INIT_COLD_JOIN,
                    record_events=True, n_dormant=6)
    o, e = SimulatedCluster(oracle, cfg), ThreadShardGroup(engine, cfg, 3)
    run_lockstep(o, e, 30, 10, "initial W=3")
    for c in (o, e):
        for m in range(39, 45):
            c.join(m, [m % 7])
    run_lockstep(o, e, 120, 30, "joins W=3")
    e.close()


def test_update_metadata(oracle, engine):
    """ClusterImpl.updateMetadata: new metadata version + incarnation bump; UPDATED events carry the new version;
    two updates of one member in one step, and one under loss."""
    cfg = SimConfig(n_members=70, record_events=True)
    o, e = pair(oracle, engine, cfg)
    run_lockstep(o, e, 15, 5, "warm")
    for c in (o, e):
        c.update_metadata(4)
        c.update_metadata(4)
        c.update_metadata(33)
    ev = run_lockstep(o, e, 60, 15, "metadata updates")
    assert {x.newMetadata for x in ev if x.isUpdated() and x.member == 4} == {2}
    for c in (o, e):
        c.set_default_loss(15)
        c.update_metadata(33)
    run_lockstep(o, e, 120, 30, "metadata update under loss")


def test_fast_config_blocks_restart_lockstep(oracle, engine):
    """MembershipProtocolTest's double partition, disabled network and restart scenarios (fast config) in lockstep:
    per-member blocks, unblockAll, a crash, a restart under a new id, a join whose only seed never started."""
    n = 7
    cc = ClusterConfig(seedMembers=[0, 1, 2, 3], syncInterval=500, syncTimeout=100, pingInterval=200,
                       pingTimeout=100, metadataTimeout=100)
    cfg = SimConfig(n_members=n, cluster=cc, init_mode=_abi.INIT_COLD_JOIN, tick_ms=10, record_events=True,
                    n_dormant=3)
    o, e = pair(oracle, engine, cfg)
    run_lockstep(o, e, 100, 20, "joined")
    for c in (o, e):
        c.block(1, 0, 2, 3)
        c.block(0, 1)
        c.block(2, 1)
    run_lockstep(o, e, 100, 20, "b lost")
    for c in (o, e):
        c.block(0, 2)
        c.block(2, 0)
    run_lockstep(o, e, 100, 20, "a, c lost")
    for c in (o, e):
        c.unblock_all()
    run_lockstep(o, e, 100, 20, "recovered")
    for c in (o, e):
        for m in range(4):
            c.block(m, 0, 1, 2, 3)
    run_lockstep(o, e, 100, 20, "network disabled")
    for c in (o, e):
        c.unblock_all()
        c.kill(3)
    run_lockstep(o, e, 150, 30, "recovered, 3 crashed")
    for c in (o, e):
        c.join(4, [0])
        c.join(5, [6])  # 6 never starts
    run_lockstep(o, e, 600, 50, "restart as 4, lonely 5")


@pytest.mark.parametrize("profile_all", [False, True])
def test_sampled_diff_accounting(oracle, engine, profile_all):
    """swim_counters diff_ns / diff_launches / diff_msgs cover the same launches (SWIM_FLAG_PROFILE samples ticks
    k % 10 == 0 on one GPU, PROFILE_ALL times all of them): with every launch timed, the payloads the timed launches
    streamed are exactly the payloads merged; sampled, they are the merges of the sampled ticks (the oracle's
    per-tick merge counts, tick by tick)."""
    import dataclasses
    cfg = SimConfig(n_members=600, cluster=ClusterConfig(syncInterval=1000))
    e = SimulatedCluster(engine, dataclasses.replace(cfg, profile=True, profile_all=profile_all))
    o = SimulatedCluster(oracle, cfg)
    e.step(7)  # the timed window starts mid-call (a call's first tick launches its own diff)
    o.step(7)
    b, want = e.counters(), 0
    for _ in range(3):
        e.step(20)
        for _ in range(20):
            t, before = o.tick, o.counters()["sync_merges"]
            o.step(1)
            if profile_all or t % 10 == 0:
                want += o.counters()["sync_merges"] - before
    c = e.counters()
    assert c["sync_merges"] == o.counters()["sync_merges"]
    assert c["diff_launches"] - b["diff_launches"] == (60 if profile_all else 6)
    # (SYNC_ACKs resolved from the write logs are merged without being streamed, k_ack_resolve)
    assert c["diff_msgs"] + c["ack_resolved"] - b["diff_msgs"] - b["ack_resolved"] == want
    assert c["ack_resolved"] > b["ack_resolved"]
    assert c["diff_ns"] > b["diff_ns"]
    e.close()


@pytest.mark.tape
@pytest.mark.parametrize("world", [1, 3])
def test_rumor_mode_at_scale_paths(oracle, engine, world):
    """The C5 code paths at test size: implicit views (the PRECONVERGED row and Feistel lists computed, not stored;
    SWIM_FLAG_IMPLICIT_VIEWS, forced here, always on above 65536 members) and, with events not recorded, the GOSSIP
    events hashed and counted where first receipts are applied (no receipt routing). Single GPU and 3 slot shards."""
    import dataclasses
    from swimhip.shard import ThreadShardGroup
    cfg = SimConfig(n_members=2000, mode=_abi.MODE_RUMOR, churn_per_period=20)
    o = SimulatedCluster(oracle, cfg)
    ecfg = dataclasses.replace(cfg, implicit_views=True)
    e = SimulatedCluster(engine, ecfg) if world == 1 else ThreadShardGroup(engine, ecfg, world)
    for c in (o, e):
        c.set_default_loss(5)
    run_lockstep(o, e, 200, 50, f"rumor implicit views W={world}", events=False)
    for c in (o, e):
        c.kill(7)
    run_lockstep(o, e, 100, 50, f"rumor implicit views + kill W={world}", events=False)
    for m in (0, 1999):
        assert o.lists(m)[1].tolist() == e.lists(m)[1].tolist()
        assert np.array_equal(o.row(m), e.row(m))
    assert e.counters()["events"] == o.counters()["events"] > 0
    e.close()


def test_c5_shard_fits_one_gpu(engine):
    """C5 (10^6 members, RUMOR, 1 % churn on 8 GPUs): rank 0 of 8 slot shards at full size fits one MI355X. Tables
    and lists are implicit; the holder table holds this shard's ~1/8 of the ~2.7·10^5 live rumors (40 000 slots)."""
    from swimhip.shard import ShardedCluster, ThreadExchange
    cfg = SimConfig(n_members=1_000_000, mode=_abi.MODE_RUMOR, churn_per_period=10_000, gossip_slot_cap=40_000)
    c = ShardedCluster(engine, cfg, 0, 8, _abi.TRANSPORT_HOST, exchange=ThreadExchange(8).endpoint(0))
    try:
        nbytes = c.counters()["device_bytes"]
    finally:
        c.close()
    assert nbytes < 250e9, nbytes
