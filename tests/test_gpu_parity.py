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


def test_preconverged_sync_large(oracle, engine):
    """C3-shaped at reduced N: no loss, steady state; exercises periodic SYNC / SYNC_ACK merges."""
    cfg = SimConfig(n_members=1500)
    o, e = pair(oracle, engine, cfg)
    run_lockstep(o, e, 320, 80, "sync", events=False)
