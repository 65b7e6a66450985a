"""Randomised fault schedules, engine against oracle, bit-exact after every chunk of ticks.

Each seed draws a member count, a config preset and a sequence of NetworkEmulator / lifecycle actions (loss changes,
two- and three-way partitions, heals, crashes, incarnation bumps). The golden c4 scenario found a replay bug that the
hand-written scenarios missed (a gossip swept while the member's gossip list was small looked live again once the
list grew back); this widens that net. Single-GPU and row-sharded (W = 2) engines both run."""
import numpy as np
import pytest

from swimhip import ClusterConfig, SimConfig, _abi
from swimhip.cluster import SimulatedCluster

from parity_util import run_lockstep

pytestmark = pytest.mark.gpu


def schedule(seed, fast_sync=False):
    rng = np.random.default_rng(seed)
    n = int(rng.choice([12, 24, 40, 64]))
    preset = rng.integers(3)
    cc = [ClusterConfig(seedMembers=[0]), ClusterConfig(seedMembers=[0, n - 1], syncInterval=5000),
          ClusterConfig.defaultLocalConfig().with_(seedMembers=[0, n // 2])][preset]
    slots = 0
    if fast_sync:  # SYNC every 2-5 ticks: several payloads per receiver and tick (MembershipProtocolImpl.java:456-467)
        cc = cc.with_(syncInterval=int(rng.choice([200, 300, 500])), syncTimeout=100)
        slots = 1 << 16  # every SYNC re-spreads the records the receiver lacked: many more live gossips
    cold = bool(rng.integers(2))
    cfg = SimConfig(n_members=n, cluster=cc, init_mode=_abi.INIT_COLD_JOIN if cold else _abi.INIT_PRECONVERGED,
                    record_events=True, seed=int(rng.integers(1 << 31)), list_slack=4096, pending_fetch_cap=4096,
                    gossip_slot_cap=slots)
    acts = [("run", int(rng.integers(20, 60)))]
    for _ in range(int(rng.integers(4, 8))):
        kind = rng.choice(["loss", "part2", "part3", "heal", "kill", "inc", "link", "block", "unblock", "leave"])
        if kind == "loss":
            acts.append(("loss", int(rng.choice([0, 5, 20, 50]))))
        elif kind in ("part2", "part3"):
            acts.append(("part", rng.integers(2 if kind == "part2" else 3, size=n).astype(np.uint32)))
        elif kind == "heal":
            acts.append(("heal", None))
        elif kind == "kill":
            acts.append(("kill", int(rng.integers(1, n))))
        elif kind == "inc":
            acts.append(("inc", int(rng.integers(n))))
        elif kind == "leave":
            acts.append(("leave", int(rng.integers(1, n))))
        elif kind == "link":  # a handful of per-link loss settings (NetworkEmulator.setLinkSettings)
            acts.append(("link", [(int(rng.integers(n)), int(rng.integers(n)), int(rng.choice([0, 30, 100])))
                                  for _ in range(int(rng.integers(1, 6)))]))
        elif kind == "block":  # one member's outbound links to a few others (NetworkEmulator.block)
            acts.append(("block", (int(rng.integers(n)), [int(x) for x in rng.integers(n, size=3)])))
        else:
            acts.append(("unblock", (int(rng.integers(n)), [int(x) for x in rng.integers(n, size=3)])))
        acts.append(("run", int(rng.integers(20, 200))))
    # user gossips (Cluster.spreadGossip) from a separate stream, so the fault schedules above stay as they were
    rg = np.random.default_rng(seed + 10_000)
    if cold and rg.integers(2):  # late joins: the last two members are dormant and start with their own seeds
        import dataclasses
        cfg = dataclasses.replace(cfg, n_dormant=2)
        for m in (n - 2, n - 1):
            pos = 1 + 2 * int(rg.integers(len(acts) // 2))
            acts.insert(pos, ("join", (m, [int(x) for x in rg.integers(n - 2, size=int(rg.integers(0, 3)))])))
    for _ in range(int(rg.integers(1, 4))):
        pos = 1 + 2 * int(rg.integers(len(acts) // 2))
        acts.insert(pos, ("gossip", [(int(rg.integers(n)), int(rg.integers(1 << 63))) for _ in range(int(rg.integers(1, 4)))]))
    return cfg, acts


def play(o, e, acts, where, n_dormant=0):
    dead = set()
    n = o.n
    dormant = set(range(n - n_dormant, n))
    for what, arg in acts:
        if what == "run":
            run_lockstep(o, e, arg, max(10, arg // 3), where)
            continue
        if what in ("inc", "leave") and arg in dead:
            continue
        if what == "gossip":
            arg = [(m, p) for m, p in arg if m not in dead]
        if what in ("inc", "leave", "kill") and arg in dormant:
            continue
        if what == "gossip":
            arg = [(m, p) for m, p in arg if m not in dormant]
        for c in (o, e):
            if what == "loss":
                c.set_default_loss(arg)
            elif what == "part":
                c.partition(arg)
            elif what == "heal":
                c.unblock_all()
            elif what == "kill":
                c.kill(arg)
            elif what == "inc":
                c.update_incarnation(arg)
            elif what == "leave":
                c.leave(arg)
            elif what == "link":
                for src, dst, pct in arg:
                    c.set_link_loss(src, dst, pct)
            elif what == "block":
                c.block(arg[0], *arg[1])
            elif what == "unblock":
                c.unblock(arg[0], *arg[1])
            elif what == "gossip":
                for m, p in arg:
                    c.spread_gossip(m, p)
            elif what == "join":
                c.join(arg[0], arg[1])
        if what in ("kill", "leave"):
            dead.add(arg)
        if what == "join":
            dormant.discard(arg[0])


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_single_gpu(oracle, engine, seed):
    cfg, acts = schedule(seed)
    o, e = SimulatedCluster(oracle, cfg), SimulatedCluster(engine, cfg)
    play(o, e, acts, f"fuzz seed {seed} N={cfg.n_members}", cfg.n_dormant)
    e.close()


@pytest.mark.parametrize("seed", range(200, 210))
def test_fuzz_fast_sync(oracle, engine, seed):
    """Fast SYNC presets, where a receiver often merges several payloads in one tick and an earlier one changes a
    row a later one holds at its start-of-tick value (leaves, suspicion removals, partitions)."""
    cfg, acts = schedule(seed, fast_sync=True)
    o, e = SimulatedCluster(oracle, cfg), SimulatedCluster(engine, cfg)
    play(o, e, acts, f"fast-sync fuzz seed {seed} N={cfg.n_members}", cfg.n_dormant)
    e.close()


@pytest.mark.parametrize("seed", range(100, 106))
def test_fuzz_sharded(oracle, engine, seed):
    from swimhip.shard import ThreadShardGroup
    cfg, acts = schedule(seed)
    o, e = SimulatedCluster(oracle, cfg), ThreadShardGroup(engine, cfg, 2)
    play(o, e, acts, f"fuzz seed {seed} N={cfg.n_members} W=2", cfg.n_dormant)
    e.close()
