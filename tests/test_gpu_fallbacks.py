"""The engine's exact fallback paths, forced and checked bit for bit against the oracle.

The fast structures of the engine have fixed capacities: subjects tracked per SYNC receiver and tick
(TRK), logged row writes and open snapshots of the deferred copy-on-write (ULOG, CREQ, CWMAX), the contact cache of
the infectedFrom replay (CEV), inbound SYNC messages sorted in registers (MQ) and receipts sorted in LDS (SORT_MAX).
Past them the engine takes slower exact paths, which the default sizes almost never reach at test scale. SWIM_CAPS
(include/swimhip_debug.h) lowers the capacities at create; the handle then counts every fallback it takes, and each
test requires both bit-exact lockstep with the oracle and that the fallbacks it targets fired
(MembershipProtocolImpl.java:446-467, GossipProtocolImpl.java:239-250)."""
import pytest

from swimhip import ClusterConfig, SimConfig, _abi
from swimhip.cluster import SimulatedCluster

from parity_util import run_lockstep
from test_gpu_fuzz import play, schedule

pytestmark = pytest.mark.gpu

TINY = "trk=1,ulog=1,creq=1,cwmax=1,cev=1,mq=1,sort=2,rx=1,hv=1"  # hv=1: every P4 with a receipt on a wave (k_inbox_apply)


def _engine(engine, cfg, monkeypatch, caps=TINY, shards=1):
    monkeypatch.setenv("SWIM_CAPS", caps)
    try:
        if shards == 1:
            return SimulatedCluster(engine, cfg)
        from swimhip.shard import ThreadShardGroup
        return ThreadShardGroup(engine, cfg, shards)
    finally:
        monkeypatch.delenv("SWIM_CAPS")


def _fallbacks(engine, e):
    if hasattr(e, "shards"):  # ThreadShardGroup: summed over its shard handles
        tot = {}
        for s in e.shards:
            for k, v in _abi.debug_fallbacks(engine, s._h).items():
                tot[k] = tot.get(k, 0) + v
        return tot
    return _abi.debug_fallbacks(engine, e._h)


@pytest.mark.parametrize("seed", [200, 201, 202, 203, 204, 205])
def test_tiny_caps_fast_sync_fuzz(oracle, engine, seed, monkeypatch):
    """Fast-SYNC fault schedules (several payloads per receiver and tick, senders that write their row after a
    send) with every capacity at its minimum: the whole-row SYNC walk, the lane copies of the copy-on-write, the
    list-walk selection of inbound messages, the slow contact replay and the merged receipt sort all run."""
    cfg, acts = schedule(seed, fast_sync=True)
    o, e = SimulatedCluster(oracle, cfg), _engine(engine, cfg, monkeypatch)
    play(o, e, acts, f"tiny caps, fast-sync seed {seed} N={cfg.n_members}", cfg.n_dormant)
    fb = _fallbacks(engine, e)
    assert sum(1 for v in fb.values() if v) >= 4, fb  # which ones depends on the schedule: all of them below
    assert fb["cev_slow"] > 0, fb  # cev=1: pairs with two or more cached contacts overflow to the slow path
    e.close()


@pytest.mark.tape
def test_tiny_caps_fallbacks_all_fire(oracle, engine, monkeypatch):
    """Across a few schedules every counted fallback fires at least once, each run bit-exact."""
    total = {}
    for seed in (200, 201, 206, 207, 208, 209):
        cfg, acts = schedule(seed, fast_sync=True)
        o, e = SimulatedCluster(oracle, cfg), _engine(engine, cfg, monkeypatch)
        play(o, e, acts, f"tiny caps seed {seed}", cfg.n_dormant)
        for k, v in _fallbacks(engine, e).items():
            total[k] = total.get(k, 0) + v
        e.close()
    for k in ("trk_walk", "ulog", "creq", "cwmax", "cev_slow", "mq", "sort_merge", "rx_all"):
        assert total[k] > 0, (k, total)


@pytest.mark.parametrize("seed", [210, 211])
def test_tiny_caps_sharded(oracle, engine, seed, monkeypatch):
    """The same fallbacks on two row shards (payloads received from the other shard take the whole-row walk
    without an arena copy)."""
    cfg, acts = schedule(seed, fast_sync=True)
    o, e = SimulatedCluster(oracle, cfg), _engine(engine, cfg, monkeypatch, shards=2)
    play(o, e, acts, f"tiny caps, 2 shards, seed {seed}", cfg.n_dormant)
    fb = _fallbacks(engine, e)
    assert sum(1 for v in fb.values() if v) >= 4 and fb["cev_slow"] > 0, fb
    e.close()


def test_contact_replay_default_caps(oracle, engine, monkeypatch):
    """Default capacities with fallback counting on: a small lossy cluster where most gossip pairs have logged
    contacts, so sends go through the cached isInfected replay (k_gossip_replay) and, past the cache, the slow
    path; bit-exact."""
    cfg = SimConfig(n_members=40, cluster=ClusterConfig(seedMembers=[0], syncInterval=2000), record_events=True,
                    gossip_slot_cap=1 << 14)
    o = SimulatedCluster(oracle, cfg)
    monkeypatch.setenv("SWIM_FALLBACKS", "1")
    e = SimulatedCluster(engine, cfg)
    monkeypatch.delenv("SWIM_FALLBACKS")
    for c in (o, e):
        c.set_default_loss(20)
        for m in range(0, 40, 7):
            c.update_incarnation(m)
    run_lockstep(o, e, 300, 50, "contact replay, loss 20")
    fb = _fallbacks(engine, e)
    assert fb["replay"] > 0, fb
    e.close()


def test_cold_join_inbound_burst(oracle, engine, monkeypatch):
    """A cold join where every member's initial SYNC goes to the one seed in the same tick (start0, :216-251): the
    seed merges N-1 payloads in one tick, with mq=1 selecting each next message by a list walk."""
    cfg = SimConfig(n_members=96, cluster=ClusterConfig(seedMembers=[0]), init_mode=_abi.INIT_COLD_JOIN,
                    record_events=True)
    o, e = SimulatedCluster(oracle, cfg), _engine(engine, cfg, monkeypatch)
    run_lockstep(o, e, 200, 20, "cold join burst, tiny caps")
    fb = _fallbacks(engine, e)
    assert fb["mq"] > 0 and fb["trk_walk"] > 0, fb
    e.close()
