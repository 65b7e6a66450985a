"""Worker for tests/test_gpu_sharded_rccl.py: one rank of a row-sharded simulation over the RCCL transport.

Both ranks may share one GPU: the launcher gives each rank its own NCCL_HOSTID, so RCCL treats them as two hosts and
connects them through its socket transport. Each rank compares its observers' state hashes, and rank 0 the summed
counters and the merged events, against the CPU oracle (which every rank runs on the full member range).
With "rumor" after the transport: RUMOR mode, slot-sharded (bench.py --workload c5 --gpus W): every
rank runs all members and keeps the gossips it owns; the per-observer hash words of held gossips and events add up
across ranks, and the merged GOSSIP events take their per-observer sequence in P4's gossip-id order."""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scalecube-cluster_amd"))
sys.path.insert(0, str(ROOT / "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import swimhip  # noqa: E402
from swimhip import ClusterConfig, SimConfig, _abi  # noqa: E402
from swimhip.cluster import SimulatedCluster  # noqa: E402
from swimhip.shard import GlooExchange, ShardedCluster, rccl_unique_id  # noqa: E402


def main():
    import faulthandler
    faulthandler.dump_traceback_later(150, exit=False)
    transport = sys.argv[1]
    rumor = len(sys.argv) > 2 and sys.argv[2] == "rumor"
    print(f"rank {os.environ['RANK']} start", flush=True)
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    print(f"rank {rank} pg up", flush=True)
    lib = swimhip.engine()
    _abi.bind_shard(lib)
    oracle = _abi.load(ROOT / "oracle" / "liboracle_swimref.so")
    n = 400
    cfg = SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0, n - 1]), record_events=True)
    if rumor:
        cfg = SimConfig(n_members=n, mode=_abi.MODE_RUMOR, churn_per_period=6, record_events=True)
    if transport == "rccl":
        obj = [rccl_unique_id(lib) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        e = ShardedCluster(lib, cfg, rank, world, _abi.TRANSPORT_RCCL, rccl_id=obj[0])
    else:
        e = ShardedCluster(lib, cfg, rank, world, _abi.TRANSPORT_HOST, exchange=GlooExchange())
    o = SimulatedCluster(oracle, cfg)
    print(f"rank {rank} shard {e.lo}..{e.hi} created", flush=True)
    t0 = time.time()
    plan = [("loss", 10), ("run", 50), ("kill", 7), ("kill", 399), ("inc", 100), ("run", 50), ("loss", 0),
            ("run", 25)]
    if rumor:
        plan[4] = ("gossip", 17)
    for what, arg in plan:
        if what == "run":
            done = 0
            while done < arg:
                o.step(25)
                e.step(25)
                done += 25
                print(f"rank {rank} tick {o.tick} {time.time() - t0:.1f}s exchange "
                      f"{e.counters()['exchange_ns'] * 1e-9:.1f}s", flush=True)
                ho, he = o.state_hash(), e.state_hash()
                if rumor:  # replicated words equal on every rank; held gossips and events summed over ranks
                    part = torch.tensor(he[:, 3:5].astype(np.int64))
                    dist.all_reduce(part)
                    he = he.copy()
                    he[:, 3:5] = part.numpy().astype(np.uint64)
                    assert np.array_equal(ho, he), f"rank {rank} tick {o.tick}: slot-sharded state hash differs"
                else:
                    lo, hi = e.lo, e.hi
                    assert np.array_equal(ho[lo:hi], he[lo:hi]), f"rank {rank} tick {o.tick}: state hash differs"
                    assert not he[:lo].any() and not he[hi:].any()
                ce = e.counters()
                keys = ["record_compares", "row_writes", "messages", "gossip_messages", "events", "messages_lost",
                        "gossips_created", "sync_merges"]
                t = torch.tensor([ce[k] for k in keys], dtype=torch.int64)
                dist.all_reduce(t)
                co = o.counters()
                assert t.tolist() == [co[k] for k in keys], f"tick {o.tick}: counters {t.tolist()} vs {co}"
        elif what == "loss":
            o.set_default_loss(arg)
            e.set_default_loss(arg)
        elif what == "kill":
            o.kill(arg)
            e.kill(arg)
        elif what == "gossip":
            o.spread_gossip(arg, 99)
            e.spread_gossip(arg, 99)
        elif what == "inc":
            o.update_incarnation(arg)
            e.update_incarnation(arg)
    mine = [(x.tick, x.observer, x.seq, x.type, x.member, x.oldMetadata, x.newMetadata, x.gossipCounter)
            for x in e.events()]
    allev = [None] * world
    dist.all_gather_object(allev, mine)
    if rank == 0:
        if rumor:  # per-observer sequence in (tick, origin, gossip counter) order, as ThreadShardGroup.events
            ev = sorted((x for part in allev for x in part), key=lambda x: (x[0], x[1], x[4], x[7]))
            cnt = {}
            merged = []
            for x in ev:
                cnt[x[1]] = cnt.get(x[1], -1) + 1
                merged.append((x[0], x[1], cnt[x[1]]) + x[3:7])
            merged.sort()
        else:
            merged = sorted(x[:7] for part in allev for x in part)
        want = [(x.tick, x.observer, x.seq, x.type, x.member, x.oldMetadata, x.newMetadata) for x in o.events()]
        assert merged == want, f"events differ: {len(merged)} vs {len(want)}"
        print(f"sharded {transport}{' rumor' if rumor else ''} W={world}: {o.tick} ticks bit-exact, {len(want)} events",
              flush=True)
    e.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
