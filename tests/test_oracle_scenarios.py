"""The reference's behavioural tests restated on the deterministic harness, run against the CPU oracle.

The reference tests use wall-clock sleeps on loopback TCP and assert eventual state. Here the same member counts,
configs and fault matrices run on virtual time. The eventual-state assertions are the reference's own. Reference file:line
on every test. tick_ms = 10 for the fast test configs (ping 200 / 100 ms), so the 4-hop ping-req chain fits the
ping-req timeout as it does on loopback.
"""
import numpy as np
import pytest

from swimhip import ClusterConfig, SimConfig, _abi
from swimhip.cluster import SimulatedCluster

# MembershipProtocolTest.testConfig (:545-554): sync 500 / 100, ping 200 / 100, metadata 100; seeds = every member
def mp_config(n, **kw):
    cc = ClusterConfig(seedMembers=list(range(n)), syncInterval=500, syncTimeout=100, pingInterval=200,
                       pingTimeout=100, metadataTimeout=100)
    return SimConfig(n_members=n, cluster=cc, init_mode=_abi.INIT_COLD_JOIN, tick_ms=10, record_events=True, **kw)


def ticks_for_seconds(sec, tick_ms=10):
    return int(sec * 1000 // tick_ms)


def trusted(c, o):
    return sorted(c.trusted(o))


def suspected(c, o):
    return sorted(c.suspected(o))


def test_initial_phase_ok(oracle):  # MembershipProtocolTest.testInitialPhaseOk (:57-81)
    c = SimulatedCluster(oracle, mp_config(3))
    c.step(ticks_for_seconds(1))
    for o in range(3):
        assert trusted(c, o) == [0, 1, 2] and suspected(c, o) == []


def test_network_partition_then_recovery(oracle):  # testNetworkPartitionThenRecovery (:83-129)
    c = SimulatedCluster(oracle, mp_config(3))
    c.step(ticks_for_seconds(3))
    c.partition(np.arange(3, dtype=np.uint32))  # each member blocks the other two
    susp_sec = 5 * 2 * 200 // 1000  # ClusterMath.suspicionTimeout(5, 3, 200) / 1000
    c.step(ticks_for_seconds(susp_sec + 2))
    for o in range(3):
        assert trusted(c, o) == [o] and suspected(c, o) == []
    c.unblock_all()
    c.step(ticks_for_seconds(500 * 2 / 1000))
    for o in range(3):
        assert trusted(c, o) == [0, 1, 2] and suspected(c, o) == []


def test_long_network_partition_no_recovery(oracle):  # testLongNetworkPartitionNoRecovery (:313-366)
    c = SimulatedCluster(oracle, mp_config(4))
    c.step(ticks_for_seconds(1))
    for o in range(4):
        assert trusted(c, o) == [0, 1, 2, 3]
    c.partition(np.array([0, 0, 1, 1], dtype=np.uint32))
    c.step(ticks_for_seconds(2))
    assert trusted(c, 0) == [0, 1] and suspected(c, 0) == [2, 3]
    assert trusted(c, 2) == [2, 3] and suspected(c, 2) == [0, 1]
    susp_sec = 5 * 3 * 200 // 1000  # suspicionTimeout(5, 4, 200)
    c.step(ticks_for_seconds(susp_sec + 1))
    for o, mine in ((0, [0, 1]), (1, [0, 1]), (2, [2, 3]), (3, [2, 3])):
        assert trusted(c, o) == mine and suspected(c, o) == []


def test_member_lost_network_then_recover(oracle):  # testMemberLostNetworkThenRecover (:131-185)
    c = SimulatedCluster(oracle, mp_config(3))
    c.step(ticks_for_seconds(1))
    c.partition(np.array([0, 1, 0], dtype=np.uint32))  # b loses the network: {b}, {a, c}
    c.step(ticks_for_seconds(1))
    assert trusted(c, 0) == [0, 2] and suspected(c, 0) == [1]
    assert trusted(c, 1) == [1] and suspected(c, 1) == [0, 2]
    c.unblock_all()
    c.step(ticks_for_seconds(2))
    for o in range(3):
        assert trusted(c, o) == [0, 1, 2] and suspected(c, o) == []


# FailureDetectorTest (:52-101): pingReqMembers 2, ping 200 / 100 ms, fixed membership
def fd_config(n, **kw):
    cc = ClusterConfig(pingInterval=200, pingTimeout=100, pingReqMembers=2, metadataTimeout=100)
    return SimConfig(n_members=n, cluster=cc, tick_ms=10, record_events=True, **kw)


def test_fd_all_trusted(oracle):  # FailureDetectorTest.testTrusted
    c = SimulatedCluster(oracle, fd_config(3))
    c.step(ticks_for_seconds(2))
    for o in range(3):
        assert trusted(c, o) == [0, 1, 2]
    assert c.events() == []


def test_fd_all_suspected(oracle):  # FailureDetectorTest.testSuspected: every link blocked
    c = SimulatedCluster(oracle, fd_config(3))
    c.partition(np.arange(3, dtype=np.uint32))
    c.step(ticks_for_seconds(1))
    for o in range(3):
        assert suspected(c, o) == sorted(set(range(3)) - {o})


def test_fd_trusted_despite_bad_network(oracle):  # FailureDetectorTest.testTrustedDespiteBadNetwork (:118-146)
    c = SimulatedCluster(oracle, fd_config(3))
    c.block(0, 1)  # a.networkEmulator().block(b.address()): only a -> b is cut; ping-req through c covers it
    c.step(ticks_for_seconds(2))
    for o in range(3):
        assert trusted(c, o) == [0, 1, 2]
        assert suspected(c, o) == []


def test_fd_suspected_member_with_normal_network(oracle):
    # FailureDetectorTest.testSuspectedMemberWithNormalNetworkGetsPartitioned (:240-299): a, b, c block d (outbound
    # only). d's pings reach them but every ack towards d is dropped, so d suspects all three and they suspect d.
    c = SimulatedCluster(oracle, fd_config(4))
    for src in (0, 1, 2):
        c.block(src, 3)
    c.step(ticks_for_seconds(1))
    for o in (0, 1, 2):
        assert 3 in suspected(c, o)
    assert suspected(c, 3) == [0, 1, 2]
    c.unblock_all()  # unblock d everywhere: the network recovers (:282-296)
    c.step(ticks_for_seconds(3))
    for o in range(4):
        assert sorted(c.members(o)) == [0, 1, 2, 3] and suspected(c, o) == []


def test_fd_member_status_change_after_network_recovery(oracle):
    # FailureDetectorTest.testMemberStatusChangeAfterNetworkRecovery (:303-341): a and b block each other
    c = SimulatedCluster(oracle, fd_config(2))
    c.block(0, 1)
    c.block(1, 0)
    c.step(ticks_for_seconds(1))
    assert suspected(c, 0) == [1] and suspected(c, 1) == [0]
    c.unblock(0, 1)
    c.unblock(1, 0)
    c.step(ticks_for_seconds(2))
    assert trusted(c, 0) == [0, 1] and trusted(c, 1) == [0, 1]


def test_link_loss_overrides_default_and_partition(oracle):
    """NetworkEmulator precedence: a link's custom setting replaces the default (:57-59); block() of a partition
    overwrites custom settings on cross-group links (:141-150); unblockAll clears every custom setting (:186-192)."""
    n = 6
    c = SimulatedCluster(oracle, SimConfig(n_members=n))
    c.set_default_loss(100)       # every default link is dead ...
    c.set_link_loss(0, 1, 0)      # ... except the custom 0 -> 1 and 1 -> 0
    c.set_link_loss(1, 0, 0)
    c.run_periods(3)
    ctr = c.counters()
    assert ctr["messages_lost"] < ctr["messages"]
    c.partition(np.array([0, 1, 0, 0, 0, 0], dtype=np.uint32))  # 0 and 1 now in different groups: custom dropped
    c.set_default_loss(0)
    before = c.counters()["messages_lost"]
    c.run_periods(2)
    assert c.counters()["messages_lost"] > before  # 1 is cut off from everyone
    c.unblock_all()


def test_graceful_leave_yields_removed_everywhere(oracle):
    """Cluster.shutdown() (ClusterImpl.java:297-313): leaveCluster spreads the member's own DEAD record; every other
    member emits REMOVED long before a suspicion timeout could, and the leaver stops once its gossip is swept
    (ClusterTest.testMembersAccessFromScheduler / testShutdownCluster shape, ClusterTest.java:306-373)."""
    n = 16
    c = SimulatedCluster(oracle, SimConfig(n_members=n, record_events=True))
    c.run_periods(3)
    c.leave(5)
    c.run_periods(3)  # far below the 25-period suspicion timeout
    ev = [e for e in c.events() if e.member == 5]
    assert sorted(e.observer for e in ev if e.isRemoved()) == [o for o in range(n) if o != 5]
    assert [r.status for r in c.records(5) if r.member == 5] == ["DEAD"]  # its own table keeps the DEAD record
    c.run_periods(12)  # spread 3 * bitlen(16) = 15 rounds, swept after 32 rounds (6.4 s)
    assert c.gossips(5) == []  # stopped: a stopped member holds nothing


def test_kill_yields_removed_everywhere(oracle):  # ClusterTest.testShutdownCluster... (:306-373)
    n = 16
    c = SimulatedCluster(oracle, SimConfig(n_members=n, record_events=True))
    c.run_periods(3)
    c.kill(5)
    c.run_periods(5 * 5 + 5)  # suspicionTimeout(5, 16) = 25 periods
    ev = [e for e in c.events() if e.member == 5]
    removed = sorted(e.observer for e in ev if e.isRemoved())
    assert removed == [o for o in range(n) if o != 5]
    assert all(e.oldMetadata == 0 for e in ev if e.isRemoved())  # REMOVED carries the metadata


@pytest.mark.parametrize("n,loss", [(10, 0), (10, 25), (50, 0), (50, 10), (50, 25)])
def test_gossip_dissemination(oracle, n, loss):  # GossipProtocolTest.testGossipProtocol (:108-175)
    c = SimulatedCluster(oracle, SimConfig(n_members=n, record_events=True))
    c.set_default_loss(loss)
    c.step(5)
    c.update_incarnation(0)  # spreads ALIVE(inc 1) of member 0 (updateIncarnation, :178-190)
    t0 = c.tick
    sweep_ms = 2 * (3 * int(n).bit_length() + 1) * 200  # ClusterMath.gossipTimeoutToSweep(3, n, 200)
    got = {}
    while c.tick - t0 < sweep_ms // 100:
        c.step(1)
        for o in range(1, n):
            if o not in got and (int(c.row(o)[0]) & 0xFFFFFFFF) >= 1:
                got[o] = c.tick - t0
        if len(got) == n - 1:
            break
    assert len(got) == n - 1, f"only {len(got)} of {n-1} received the gossip"
    assert max(got.values()) * 100 < sweep_ms
    ev = [e for e in c.events() if e.member == 0 and e.isUpdated()]
    per_observer = {}
    for e in ev:
        per_observer[e.observer] = per_observer.get(e.observer, 0) + 1
    assert all(v == 1 for v in per_observer.values()), "double delivery"


# GossipProtocolTest.experiments (:50-64) with mean delay 2 ms (delay is not modelled: one tick of latency); a user
# gossip (Cluster.spreadGossip -> GossipProtocolImpl.spread) from member 0. Assertions of testGossipProtocol
# (:150-175): all N-1 members receive it (listenGossips), within gossipTimeoutToSweep, and none twice.
@pytest.mark.parametrize("n,loss", [(2, 0), (3, 0), (5, 0), (10, 0), (10, 10), (10, 25), (10, 50), (50, 0), (50, 10)])
def test_user_gossip_experiments(oracle, n, loss):
    c = SimulatedCluster(oracle, SimConfig(n_members=n, record_events=True))
    c.set_default_loss(loss)
    c.step(3)
    c.spread_gossip(0, 0xC0FFEE00000000 | n)
    t0 = c.tick
    sweep_ticks = 2 * (3 * int(n).bit_length() + 1) * 2  # gossipTimeoutToSweep(3, n, 200 ms) in 100 ms ticks
    c.step(sweep_ticks + 3 * 2)  # awaitFullCompletion: lifetime plus three gossip intervals
    ev = [e for e in c.events() if e.isGossip()]
    assert all(e.member == 0 and e.payload() == 0xC0FFEE00000000 | n for e in ev)
    receivers = [e.observer for e in ev]
    assert sorted(set(receivers)) == list(range(1, n)), "not all members received the gossip"
    assert len(receivers) == len(set(receivers)), "delivered gossip twice to the same member"
    assert max(e.tick for e in ev) - t0 < sweep_ticks, "dissemination slower than the gossip timeout"


def test_user_gossips_order_and_dead_origin(oracle):
    """Two gossips of one member in one tick keep call order in their ids; a killed member's queued gossip never
    starts; swim_spread_gossip on a dead member is rejected."""
    c = SimulatedCluster(oracle, SimConfig(n_members=20, record_events=True))
    c.step(2)
    c.spread_gossip(3, 1)
    c.spread_gossip(3, 2)
    c.spread_gossip(4, 3)
    c.kill(4)
    c.step(60)
    got = {}
    for e in c.events():
        if e.isGossip():
            got.setdefault(e.payload(), set()).add(e.observer)
    assert got[1] == got[2] == set(range(20)) - {3, 4}
    assert 3 not in got
    with pytest.raises(Exception):
        c.spread_gossip(4, 9)


def test_rumor_mode_churn(oracle):
    """RUMOR mode (SEMANTICS.md §9, C5 shape): no FD / SYNC / metadata traffic; every period `churn` rumors about
    Philox-chosen members, each delivered to all N - 1 other members exactly once (GossipProtocolTest :150-175)."""
    n, churn, periods = 200, 3, 25
    c = SimulatedCluster(oracle, SimConfig(n_members=n, mode=_abi.MODE_RUMOR, churn_per_period=churn, record_events=True))
    c.run_periods(periods)
    ctr = c.counters()
    assert ctr["messages"] == 0 and ctr["sync_merges"] == 0 and ctr["record_compares"] == 0
    assert ctr["gossips_created"] == churn * periods
    got = {}
    for e in c.events():
        assert e.isGossip()
        got.setdefault((e.member, e.payload()), []).append(e.observer)
    done = [(o, p) for (o, p) in got if (p >> 32) < periods - 4]  # rumors old enough to have finished
    assert len(done) == churn * (periods - 4)
    for key in done:
        obs = got[key]
        assert sorted(obs) == sorted(set(range(n)) - {key[0]}), key
    assert all((p & 0xFFFFFFFF) != o for (o, p) in got)  # the origin is never the churned member


def test_rumor_mode_requires_preconverged(oracle):
    with pytest.raises(Exception):
        SimulatedCluster(oracle, SimConfig(n_members=10, mode=_abi.MODE_RUMOR, init_mode=_abi.INIT_COLD_JOIN))


def test_limited_seed_members(oracle):  # MembershipProtocolTest.testLimitedSeedMembers (:433-462)
    """a has no seeds, b and c seed on a, d and e seed on b; after 3 s everyone trusts everyone."""
    cfg = mp_config(5, n_dormant=5)
    c = SimulatedCluster(oracle, cfg)
    for m, seeds in [(0, []), (1, [0]), (2, [0]), (3, [1]), (4, [1])]:
        c.join(m, seeds)
    c.step(ticks_for_seconds(3))
    for o in range(5):
        assert trusted(c, o) == [0, 1, 2, 3, 4] and suspected(c, o) == []


def test_restart_failed_members(oracle):  # MembershipProtocolTest.testRestartFailedMembers (:369-430)
    """c and d stop; after the suspicion timeout a and b trust only each other; c and d restart (new ids 4 and 5, as
    the reference's restarted members get new ids) seeded on a and b, and all four trust each other."""
    c = SimulatedCluster(oracle, mp_config(6, n_dormant=2))  # members 4, 5: the restarted c, d
    c.step(ticks_for_seconds(1))
    for o in range(4):
        assert trusted(c, o) == [0, 1, 2, 3]
    c.kill(2)
    c.kill(3)
    c.step(ticks_for_seconds(1))
    for o in (0, 1):
        assert trusted(c, o) == [0, 1] and suspected(c, o) == [2, 3]
    susp_sec = 5 * 3 * 200 // 1000  # ClusterMath.suspicionTimeout(5, 4, 200) / 1000
    c.step(ticks_for_seconds(susp_sec + 1))
    for o in (0, 1):
        assert trusted(c, o) == [0, 1] and suspected(c, o) == []
    c.join(4, [0, 1])
    c.join(5, [0, 1])
    c.step(ticks_for_seconds(1))
    for o in (0, 1, 4, 5):
        assert trusted(c, o) == [0, 1, 4, 5] and suspected(c, o) == [], o


def test_join_rules(oracle):
    c = SimulatedCluster(oracle, mp_config(4, n_dormant=1))
    with pytest.raises(Exception):
        c.join(1, [0])  # not dormant
    c.step(5)
    c.join(3, [0, 0, 3, 99])  # duplicates, self and unknown ids are dropped
    with pytest.raises(Exception):
        c.join(3, [0])  # joins once
    c.step(ticks_for_seconds(1))
    assert trusted(c, 3) == [0, 1, 2, 3]
    with pytest.raises(Exception):
        SimulatedCluster(oracle, SimConfig(n_members=4, n_dormant=1))  # PRECONVERGED has no dormant members


def test_update_metadata(oracle):  # ClusterTest.testUpdateMetadata (:108-169)
    """A seed, a metadata member and ten others join; after 3 s all know the metadata member with its metadata
    (version 0); after updateMetadata every other member emits UPDATED carrying the new version and stores it."""
    n = 12
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0]), init_mode=_abi.INIT_COLD_JOIN,
                    record_events=True)
    c = SimulatedCluster(oracle, cfg)
    c.step(ticks_for_seconds(3, 100))
    for o in range(n):
        recs = {r.member: r for r in c.records(o)}
        assert 1 in recs and recs[1].has_metadata
    c.events()
    c.update_metadata(1)
    c.step(ticks_for_seconds(3, 100))
    ups = [e for e in c.events() if e.isUpdated() and e.member == 1]
    assert sorted(e.observer for e in ups) == [o for o in range(n) if o != 1]
    assert all(e.oldMetadata == 0 and e.newMetadata == 1 for e in ups)


def _check_views(c, views):
    for o, (tr, su) in views.items():
        assert trusted(c, o) == tr and suspected(c, o) == su, (o, trusted(c, o), suspected(c, o))


def test_double_partition_then_recover(oracle):  # MembershipProtocolTest.testDoublePartitionThenRecover (:188-256)
    c = SimulatedCluster(oracle, mp_config(3))
    c.step(ticks_for_seconds(1))
    _check_views(c, {o: ([0, 1, 2], []) for o in range(3)})
    c.block(1, 0, 2)  # b lost the network
    c.block(0, 1)
    c.block(2, 1)
    c.step(ticks_for_seconds(1))
    _check_views(c, {0: ([0, 2], [1]), 1: ([1], [0, 2]), 2: ([0, 2], [1])})
    c.block(0, 2)  # a and c lost the network
    c.block(2, 0)
    c.step(ticks_for_seconds(1))
    _check_views(c, {0: ([0], [1, 2]), 1: ([1], [0, 2]), 2: ([2], [0, 1])})
    c.unblock_all()
    c.step(ticks_for_seconds(1))
    _check_views(c, {o: ([0, 1, 2], []) for o in range(3)})


def test_network_disabled_then_recovered(oracle):  # MembershipProtocolTest.testNetworkDisabledThenRecovered (:258-311)
    c = SimulatedCluster(oracle, mp_config(3))
    c.step(ticks_for_seconds(1))
    _check_views(c, {o: ([0, 1, 2], []) for o in range(3)})
    for m in range(3):
        c.block(m, 0, 1, 2)  # block(members): every link, including to itself
    c.step(ticks_for_seconds(1))
    _check_views(c, {0: ([0], [1, 2]), 1: ([1], [0, 2]), 2: ([2], [0, 1])})
    c.unblock_all()
    c.step(ticks_for_seconds(1))
    _check_views(c, {o: ([0, 1, 2], []) for o in range(3)})


def test_fd_status_change_after_member_restart(oracle):  # FailureDetectorTest.testStatusChangeAfterMemberRestart
    """(:345-401) a, b, x; x stops, then a new process x' (new id) starts seeded on a: a and b see x suspected, then
    x' trusted. (Later, the cold-join ALIVE gossips about x that are still circulating re-add x after its removal, with
    no ADDED event because its metadata cannot be fetched: the reference's own zombie behaviour, not asserted there.)"""
    c = SimulatedCluster(oracle, mp_config(4, n_dormant=1))  # member 3 = x'
    c.step(ticks_for_seconds(1))
    c.kill(2)
    c.step(ticks_for_seconds(1))
    for o in (0, 1):
        assert 2 in suspected(c, o)
    c.join(3, [0])
    c.step(ticks_for_seconds(1))
    for o in (0, 1, 3):
        assert 3 in trusted(c, o) and 3 not in suspected(c, o)


def test_join_seed_cluster_with_no_existing_seed_member(oracle):  # ClusterTest (:376-392)
    """A member whose only seed does not exist (a dead id) starts alone: the initial sync fails and it keeps running
    with itself as the only member."""
    cc = ClusterConfig(seedMembers=[0], syncInterval=500, syncTimeout=100, pingInterval=200, pingTimeout=100,
                       metadataTimeout=100)
    c = SimulatedCluster(oracle, SimConfig(n_members=3, cluster=cc, init_mode=_abi.INIT_COLD_JOIN, tick_ms=10,
                                           n_dormant=2, record_events=True))
    c.join(2, [1])  # member 1 never starts: a seed address with no member behind it
    c.step(ticks_for_seconds(2))
    assert trusted(c, 2) == [2] and suspected(c, 2) == []
    assert trusted(c, 0) == [0]


def test_fd_trusted_despite_different_ping_timings(oracle):
    # FailureDetectorTest.testTrustedDespiteDifferentPingTimings (:150-178): a runs the fast test config, b and c
    # the default FD timings (1000 / 500 ms); every member keeps the other two trusted
    c = SimulatedCluster(oracle, fd_config(3))
    for m in (1, 2):
        c.set_member_config(m, ClusterConfig(pingInterval=1000, pingTimeout=500))
    c.step(ticks_for_seconds(5))
    for o in range(3):
        assert trusted(c, o) == [0, 1, 2] and suspected(c, o) == []
    assert c.events() == []


def test_fd_suspected_member_with_bad_network(oracle):
    # FailureDetectorTest.testSuspectedMemberWithBadNetworkGetsPartitioned (:181-237): a blocks its traffic to every
    # member; a suspects b, c, d and they suspect a. Then a.networkEmulator().unblockAll(): a's own settings only
    # (per-link unblock), and after 4 s every member trusts every other again.
    c = SimulatedCluster(oracle, fd_config(4))
    c.block(0, 0, 1, 2, 3)
    c.step(ticks_for_seconds(1))
    assert suspected(c, 0) == [1, 2, 3]
    for o in (1, 2, 3):
        assert suspected(c, o) == [0]
    c.unblock(0, 0, 1, 2, 3)
    c.step(ticks_for_seconds(4))
    for o in range(4):
        assert trusted(c, o) == [0, 1, 2, 3] and suspected(c, o) == []


def test_sync_groups_do_not_merge(oracle):
    # MembershipProtocolImpl.checkSyncGroup (:320-331,431-437): a member ignores SYNC / SYNC_ACK data of another
    # syncGroup. Cold join through seed 0: members 4..5 are in group "other", so their initial syncs with seed 0 time
    # out unanswered and seed 0 ignores theirs; they learn the cluster only through gossip and FD-triggered traffic.
    import dataclasses
    n = 6
    cfg = dataclasses.replace(mp_config(n), cluster=ClusterConfig(
        seedMembers=[0], syncInterval=500, syncTimeout=100, pingInterval=200, pingTimeout=100, metadataTimeout=100))
    same = SimulatedCluster(oracle, cfg)
    split = SimulatedCluster(oracle, cfg)
    for m in (4, 5):
        split.set_member_config(m, ClusterConfig(pingInterval=200, pingTimeout=100, syncGroup="other"))
    for c in (same, split):
        c.step(ticks_for_seconds(3))
    for o in range(n):
        assert sorted(same.members(o)) == list(range(n))
    assert split.members(4) == [4] and split.members(5) == [5]  # no SYNC of theirs was ever merged, nor answered
    for o in range(4):
        assert 4 not in split.members(o) and 5 not in split.members(o)
