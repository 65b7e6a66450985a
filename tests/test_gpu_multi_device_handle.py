"""One handle over several GPUs (swim_config.n_gpus > 1): swim_create builds the row-sharded shards
itself, one per device, and every ABI call is forwarded. A Java or ctypes host keeps a single handle and
one thread, as with one GPU. On a node with fewer devices than n_gpus (the single-GPU test box) the shards share the
device and exchange through host memory inside the process; on 8 GPUs they use RCCL. Bit-exact against the oracle,
through the plain C ABI (SimulatedCluster: one handle)."""
import dataclasses

import numpy as np
import pytest

from swimhip import ClusterConfig, SimConfig, _abi
from swimhip.cluster import SimulatedCluster

from parity_util import run_lockstep

pytestmark = pytest.mark.gpu


def pair(oracle, engine, cfg, gpus):
    return SimulatedCluster(oracle, cfg), SimulatedCluster(engine, dataclasses.replace(cfg, n_gpus=gpus))


@pytest.mark.parametrize("gpus", [2, 3])
def test_c1_cold_join_kill(oracle, engine, gpus):
    cfg = SimConfig(n_members=64, cluster=ClusterConfig(seedMembers=[0]), init_mode=_abi.INIT_COLD_JOIN,
                    record_events=True)
    o, e = pair(oracle, engine, cfg, gpus)
    run_lockstep(o, e, 100, 10, f"C1 join n_gpus={gpus}")
    for c in (o, e):
        c.kill(63)
    ev = run_lockstep(o, e, 400, 50, f"C1 kill n_gpus={gpus}")
    assert sorted(x.observer for x in ev if x.isRemoved() and x.member == 63) == list(range(63))
    e.close()


def test_loss_partition_gossip_configs(oracle, engine):
    n = 90
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0, 60]), record_events=True)
    o, e = pair(oracle, engine, cfg, 2)
    for c in (o, e):
        c.set_member_config(5, ClusterConfig(pingInterval=500, pingTimeout=200, pingReqMembers=1))
        c.set_default_loss(10)
    run_lockstep(o, e, 100, 20, "loss 10")
    g = np.array([0] * 45 + [1] * 45, dtype=np.uint32)
    for c in (o, e):
        c.partition(g)
        c.spread_gossip(3, 0xABCD)
        c.leave(70)
        c.update_metadata(10)
    run_lockstep(o, e, 300, 50, "partition + gossip + leave + metadata")
    for c in (o, e):
        c.unblock_all()
    run_lockstep(o, e, 300, 50, "healed")
    lo, hi = _abi_range(e)
    assert (lo, hi) == (0, n)
    for obs in (0, 44, 45, 89):  # readback from the owning shard
        assert np.array_equal(o.row(obs), e.row(obs))
        fo, go, co = o.lists(obs)
        fe, ge, ce = e.lists(obs)
        assert np.array_equal(fo, fe) and np.array_equal(go, ge) and co == ce
        assert o.gossips(obs) == e.gossips(obs)
    e.close()


def _abi_range(c):
    import ctypes as C
    _abi.bind_shard(c.lib)
    lo, hi = C.c_uint32(), C.c_uint32()
    assert c.lib.swim_shard_range(c._h, C.byref(lo), C.byref(hi)) == 0
    return lo.value, hi.value


def test_rumor_mode(oracle, engine):
    cfg = SimConfig(n_members=200, mode=_abi.MODE_RUMOR, churn_per_period=3, record_events=True)
    o, e = pair(oracle, engine, cfg, 2)
    for c in (o, e):
        c.set_default_loss(10)
    run_lockstep(o, e, 150, 50, "rumor n_gpus=2")
    e.close()


@pytest.mark.parametrize("gpus", [1, 2])
def test_drain_small_cap(oracle, engine, gpus):
    """swim_drain_events with a cap far below the buffered count: every call returns the next events in order and
    the per-observer seq numbers neither skip nor repeat (slot-sharded RUMOR group: they are renumbered once)."""
    cfg = SimConfig(n_members=120, mode=_abi.MODE_RUMOR, churn_per_period=4, record_events=True)
    o, e = pair(oracle, engine, cfg, gpus)
    for part in range(3):
        o.step(40)
        e.step(40)
        eo, ee = o.events(), e.events(cap=7)  # several small drains per call, leftovers carried between them
        assert eo == ee, f"part {part}: {len(eo)} oracle vs {len(ee)} engine events"
    e.close()
