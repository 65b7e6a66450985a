#!/usr/bin/env python3
"""bench.py — member·periods/sec of the gfx950 SWIM engine (libswimhip) on the BASELINE.json headline config.

Workload (BASELINE.json configs[2], the config the metric "member·periods/sec at 100k members" is quoted on): 100 000
members with full membership views, PRECONVERGED (every row ALIVE inc 0, shuffled FD and gossip lists), the default
ClusterConfig (ping 1 s / 500 ms, ping-req 3, gossip 200 ms x fanout 3 x repeat 3, SYNC every 30 s), no loss. One
"step" = one FD period (pingInterval = 10 ticks of 100 ms) for every member. In this steady state every member pings
one peer per period, and periodic SYNC / SYNC_ACK anti-entropy streams whole 100k-record payloads against whole
receiver rows (N/30 syncs per period in each direction), so the dominant kernel is k_sync_diff. It is HBM-bound with
no dense math, so no MFMA: on one GPU it compares the 8-bit shadows of the record keys (2 B of algorithmic traffic
per record compare, payload + receiver; an escaped key past incarnation 62 is compared on its 4-B key), on a row
shard the 4-B keys (8 B per compare; SURVEY.md §8d priced it at 16 B for 8-B keys).

With N=1, all 100k members run on one MI355X (about 206 GB of HBM). With --gpus N under torch.distributed.run, the
SAME 100k-member cluster is row-sharded: rank r owns observers [r N/W, (r+1) N/W) and its rows (about 206/W GB), the
gossip plane is replicated, and every tick the shards exchange gossip records and SYNC payloads with RCCL send/recv
groups over xGMI inside libswimhip (include/swimhip_shard.h). Total work is fixed as N grows, so
scaling is "strong" and `value` is the whole cluster's member·periods/s. torch.distributed (gloo) only bootstraps:
it broadcasts the RCCL unique id, runs the barriers and takes the max time over ranks.

The JSON line also carries:
  roofline      k_sync_diff algorithmic bytes (the key bytes the engine counts per streamed payload: 2 B or 8 B x N,
                swim_counters.diff_key_bytes) / its HIP-event time, against 8 TB/s; traffic = measured HBM bytes per
                launch from a committed rocprofv3 PMC summary when available (profiles/), else null.
  cpu_baseline  the CPU oracle (oracle/swimref.cpp, a port) on a bounded sample: same workload shape at 10k members,
                timed here on the host on all its cores (worker threads over observer ranges, at most 16) and on one.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "scalecube-cluster_amd"))

HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
HBM_STREAM_GBPS = 6290.0  # measured streaming ceiling (MI355X_MICROARCH.md: float4 copy, 79 % of spec)
BASELINE_WORKLOAD = "C3: 100k members, full views, preconverged, default ClusterConfig, no loss"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30, help="timed FD periods")
    p.add_argument("--warmup", type=int, default=3, help="untimed FD periods")
    p.add_argument("--workload", choices=["c3", "c3dyn", "c2", "c5"], default="c3",
                   help="c3 (default, the headline): 100k full views; c3dyn: the same with membership evolution "
                        "(--updates incarnation bumps per period, MembershipProtocolImpl.updateIncarnation); "
                        "c2: 10k full views with 5%% loss; c5: rumor-only (SWIM_MODE_RUMOR) with 1%% churn per period")
    p.add_argument("--updates", type=int, default=1, help="c3dyn: updateIncarnation calls per period")
    p.add_argument("--members", type=int, default=None, help="default: 100k (c3, c5), 10k (c2)")
    p.add_argument("--loss", type=int, default=None, help="default: 5 (c2), 0 otherwise")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-members", type=int, default=None, help="default: the workload's size if host RAM allows")
    p.add_argument("--cpu-periods", type=int, default=120)
    p.add_argument("--transport", choices=["rccl", "host"], default="rccl", help="N>1 shard exchange")
    p.add_argument("--no-events", action="store_true", help="no per-kernel HIP events (roofline unavailable)")
    p.add_argument("--rehearse-shard", type=int, default=0, metavar="W",
                   help="c5 only: run rank 0 of W slot shards on this GPU alone, the other shards' gossip-count "
                        "deltas taken as zero (a per-shard timing rehearsal of the W-GPU run, not its results)")
    p.add_argument("--slots", type=int, default=0, help="gossip slots per shard (0: the engine's default)")
    p.add_argument("--ring", type=int, default=0, help="receipt-ring entries per member (0: the engine's default)")
    p.add_argument("--churn", type=int, default=0, help="c5: churn rumors per period (default: 1 %% of the members)")
    p.add_argument("--rehearse-one-gpu", action="store_true",
                   help="N>1 on a single GPU (functional rehearsal only): every rank uses device 0 and gets its own "
                        "NCCL_HOSTID, so RCCL connects the ranks through its socket transport")
    return p.parse_args()


def traffic_from_profiles(n_members):
    """HBM bytes per k_sync_diff launch from a committed rocprofv3 PMC summary for this member count, if present."""
    f = ROOT / "profiles" / "pmc_sync_diff_k8.json"  # measured with the 8-bit shadow key plane
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        if d.get("members") == n_members:
            return d.get("bytes_per_launch")
    except Exception:
        pass
    return None


def whole_step_pmc(workload, n_members):
    """Whole-step HBM bytes per period from a committed PMC summary (tools/make_profiles.py wholestep), if present."""
    f = ROOT / "profiles" / "pmc_whole_step.json"
    try:
        d = json.loads(f.read_text()).get(workload)
        if d and d.get("members") == n_members:
            return {"bytes": d["bytes_per_period"], "source": f"profiles/pmc_whole_step.json ({d['round']})"}
    except Exception:
        pass
    return None


def mem_available():
    try:
        for line in open("/proc/meminfo"):
            if line.startswith("MemAvailable:"):
                return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 0


def workload_config(a, SimConfig, _abi, members, **kw):
    if a.slots:
        kw["gossip_slot_cap"] = a.slots
    if a.ring:
        kw["gossip_ring_cap"] = a.ring
    if a.workload == "c5":
        return SimConfig(n_members=members, mode=_abi.MODE_RUMOR, churn_per_period=a.churn or max(1, members // 100),
                         **kw)
    return SimConfig(n_members=members, **kw)


def _oracle_rate(a, lib, members, periods, threads):
    from swimhip import SimConfig, SimulatedCluster, _abi
    os.environ["SWIMREF_THREADS"] = str(threads)  # read when the oracle handle is created
    c = SimulatedCluster(lib, workload_config(a, SimConfig, _abi, members))
    if a.loss:
        c.set_default_loss(a.loss)
    rng = __import__("random").Random(0x5EED)

    def run(n):
        for _ in range(n):
            for _ in range(a.updates if a.workload == "c3dyn" else 0):
                c.update_incarnation(rng.randrange(members))
            c.run_periods(1)

    run(1)
    t0 = time.perf_counter()
    run(periods)
    dt = time.perf_counter() - t0
    c.close()
    return members * periods / dt, dt


def cpu_baseline(a, members, periods):
    """Bounded CPU sample: the oracle on the same workload shape at `members` members, on all host cores (observer
    ranges per worker thread, SWIMREF_THREADS) and, for reference, on one core."""
    from swimhip import _abi
    lib_path = ROOT / "oracle" / "liboracle_swimref.so"
    if not lib_path.exists():
        import subprocess
        subprocess.check_call(["make", "-s", "-C", str(ROOT / "oracle")])
    lib = _abi.load(lib_path)
    cores = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count() or 1))
    one_members = min(members, 10_000)  # one core: the setup alone is O(N^2) single-threaded work
    one, dt1 = _oracle_rate(a, lib, one_members, max(1, min(periods, 120) // 4), 1)
    allc, dtn = _oracle_rate(a, lib, members, periods, cores)
    os.environ.pop("SWIMREF_THREADS", None)
    full = "the headline size" if members == a.members else (
        f"reduced N: the oracle holds ~20 B per member pair ({20 * a.members ** 2 / 1e9:.0f} GB of host RAM at "
        f"{a.members}), more than this host had available")
    note = {"c3": f"{full}; per-member work grows ~linearly with N (SYNC payloads)",
            "c3dyn": f"{full}; {a.updates} updateIncarnation per period as on the GPU",
            "c2": "per-member gossip load grows ~N (SYNC re-spread storm), so at 10k it is far slower per member·period",
            "c5": "per-member rumor load grows ~N at 1 % churn, so at full N it is slower per member·period"}[a.workload]
    return {"value": allc, "unit": "member·periods/s", "cores": cores, "kind": "port",
            "single_core_value": one, "single_core_members": one_members,
            "sample": f"oracle/swimref.cpp, {members} members (same {a.workload.upper()} shape), {periods} "
                      f"periods after 1 warm-up period on {cores} worker threads ({dtn:.1f} s), and "
                      f"{max(1, min(periods, 120) // 4)} periods at {one_members} members on one core ({dt1:.1f} s); "
                      f"{note}"}


def workload_name(a, n):
    if a.workload == "c3dyn":
        return (f"C3 with membership evolution: {n} members, full views, preconverged, {a.updates} "
                f"updateIncarnation per period (gossip, SYNC re-spread, UPDATED events, metadata fetches)")
    if a.workload == "c3":
        return BASELINE_WORKLOAD if (n == 100_000 and not a.loss) else f"{n} members, full views, loss {a.loss}%"
    if a.workload == "c2":
        return f"C2: {n} members, full views, preconverged, loss {a.loss}%"
    what = "C5" if n >= 1_000_000 else "C5 (reduced N)"
    shard = (f"; rank 0 of {a.rehearse_shard} slot shards alone (the other shards' gossip-count deltas zero: a "
             f"per-shard timing rehearsal, not the {a.rehearse_shard}-GPU result)") if a.rehearse_shard > 1 else ""
    return (f"{what}: {n} members, rumor-only, {a.churn or max(1, n // 100)} churn rumors per period, loss "
            f"{a.loss}%{shard}")


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.rehearse_one_gpu:
        local = 0
        os.environ["NCCL_HOSTID"] = f"swim-rehearsal-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    import torch

    dist = None
    import swimhip
    from swimhip import SimConfig, _abi

    if a.members is None:
        a.members = 10_000 if a.workload == "c2" else 100_000
    if a.loss is None:
        a.loss = 5 if a.workload == "c2" else 0
    cfg = workload_config(a, SimConfig, _abi, a.members, device=local, profile=not a.no_events)
    if a.rehearse_shard > 1:
        if a.workload != "c5" or world != 1:
            raise SystemExit("--rehearse-shard needs --workload c5 on one GPU")
        from swimhip.shard import LoneExchange, ShardedCluster
        os.environ["SWIM_LONE_SHARD"] = "1"  # the engine skips the (simulated) exchange altogether
        lib = swimhip.engine()
        c = ShardedCluster(lib, cfg, 0, a.rehearse_shard, _abi.TRANSPORT_HOST, exchange=LoneExchange(a.rehearse_shard))
    elif world > 1:
        import torch.distributed as dist
        from swimhip.shard import GlooExchange, ShardedCluster, rccl_unique_id
        dist.init_process_group("gloo")
        lib = swimhip.engine()
        _abi.bind_shard(lib)
        if a.transport == "rccl":
            obj = [rccl_unique_id(lib) if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            c = ShardedCluster(lib, cfg, rank, world, _abi.TRANSPORT_RCCL, rccl_id=obj[0])
        else:
            c = ShardedCluster(lib, cfg, rank, world, _abi.TRANSPORT_HOST, exchange=GlooExchange())
    else:
        c = swimhip.cluster(cfg)
    if a.loss:
        c.set_default_loss(a.loss)
    rng = __import__("random").Random(0x5EED)

    def run(periods):
        if a.workload != "c3dyn":
            c.run_periods(periods)
            return
        for _ in range(periods):  # members chosen on the host: every rank makes the same calls
            for _ in range(a.updates):
                c.update_incarnation(rng.randrange(a.members))
            c.run_periods(1)

    run(a.warmup)
    base = c.counters()

    def barrier():
        c.sync()
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    barrier()
    t0 = time.perf_counter()
    run(a.steps)
    barrier()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ctr = c.counters()
    d = {k: ctr[k] - base[k] for k in ctr}

    if rank == 0:
        n = a.members
        ticks_per_period = cfg.cluster.pingInterval // cfg.tick_ms
        merges = d["sync_merges"]
        diff_s = d["diff_ns"] * 1e-9
        launches = max(1, d["diff_launches"])
        # the engine counts the key bytes its timed k_sync_diff launches compared (every 10th tick on one GPU, every
        # tick on a row shard): 2 x 1 B per subject for a payload streamed from the 8-bit shadow plane, 2 x 4 B for
        # the others; SYNC_ACKs resolved from write logs are not streamed, so they are not priced here
        timed_bytes = d["diff_key_bytes"]
        bytes_per_launch = timed_bytes / launches
        achieved = timed_bytes / diff_s / 1e9 if diff_s > 0 else 0.0
        # whole-step algorithmic bytes, SURVEY.md §8d with 4-B record keys (B = 8R + 8W + 32M + 0.375G + 24E), with R's
        # SYNC part priced as the engine reads it: the key bytes k_sync_diff compared per streamed payload (above), and
        # for a SYNC_ACK resolved from write logs (k_ack_resolve) at most 3 x 16 subjects x 8 B; every other record
        # compare at 8 B. (R counts the sender's table size per merged payload, N in these preconverged workloads.)
        resolved = d["ack_resolved_total"]
        r_other = max(0, d["record_compares"] - n * merges)
        B = (d["diff_key_bytes_total"] + 8 * 48 * resolved + 8 * r_other + 8 * d["row_writes"] + 32 * d["messages"]
             + 0.375 * d["gossip_messages"] + 24 * d["events"])
        line = {
            "metric": "member·periods/sec at 100k members (whole node); achieved HBM GB/s",
            "value": n * a.steps / dt,
            "unit": "member·periods/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": dt * 1e3 / a.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            # record keys are u32 `inc << 2 | status`: incarnations are capped at 2^30 - 1 (Java int: 2^31 - 1), past
            # which the engine raises SWIM_ECAPACITY (SEMANTICS.md §8); the diff compares their exact 8-bit shadows
            # (a key past 0xFE escapes to its u32 compare); list entries are u32 member ids
            "dtype": ("u8 key shadows, exact (u32 record key inc<<2|status: 30-bit incarnation cap)" if world == 1
                      else "u32 (record key inc<<2|status: 30-bit incarnation cap)"),
            "data": "synthetic (PRECONVERGED full views, seeded Philox selector)",
            "config": {"workload": workload_name(a, n),
                       "members": n, "periods_per_step": 1, "ticks_per_period": ticks_per_period,
                       "parallelism": (f"{'slot' if a.workload == 'c5' else 'row'}-sharded x{world} ({a.transport})"
                                       if world > 1 else "single-gpu")},
            "roofline": {"bound": "hbm", "kernel": "k_sync_diff", "achieved": achieved, "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBPS,
                         "frac_of_measured_stream_ceiling": achieved / HBM_STREAM_GBPS,
                         "algorithmic_bytes_per_launch": bytes_per_launch,
                         "avg_launch_us": diff_s * 1e6 / launches,
                         # the same launches priced by SURVEY.md §8d's model (16 B per record compare: 8-B keys read
                         # on both sides), which predates the 4-B key plane and its 2-B shadow: above 1 means the
                         # engine reads fewer bytes per compare than that model assumes, not that it skips compares
                         "survey_8d_model": {
                             "bytes_per_compare": 16,
                             "bytes_per_launch": 16 * n * d["diff_msgs"] / launches,
                             "achieved": 16 * n * d["diff_msgs"] / diff_s / 1e9 if diff_s > 0 else 0.0,
                             "frac": (16 * n * d["diff_msgs"] / diff_s / 1e9 / HBM_PEAK_GBPS) if diff_s > 0 else 0.0},
                         "traffic": traffic_from_profiles(n) if world == 1 else None,
                         "traffic_source": "committed rocprofv3 PMC summary profiles/pmc_sync_diff_k8.json (FETCH_SIZE x 2 "
                                           "+ WRITE_SIZE per launch), not measured in this run"},
            # the engine times a sample of the launches (every 10th tick on one GPU): average x launches per period
            "kernel_time_share": {"k_sync_diff": diff_s / launches * ticks_per_period * a.steps / dt},  # others: profiles/*kernel_stats*
            "whole_step_algorithmic_GBps": B / dt / 1e9,
            "whole_step_algorithmic_bytes_per_period": B / a.steps,
            # whole-step HBM bytes per period measured by rocprofv3 PMC (FETCH_SIZE x 2 + WRITE_SIZE over every kernel,
            # the difference of two runs of different lengths): read from the committed profiles/, not this run
            "whole_step_pmc_bytes_per_period_committed": whole_step_pmc(a.workload, n) if world == 1 else None,
            "counters": {k: d[k] for k in ("record_compares", "row_writes", "messages", "gossip_messages", "events",
                                           "sync_merges", "diff_msgs_total", "ack_resolved_total",
                                           "diff_key_bytes_total")},
            "device_bytes": ctr["device_bytes"],
            # since the handle was created (warm-up included): a profiler pass over the whole process prices its
            # k_sync_diff traffic against these key bytes (tools/make_profiles.py)
            "run_totals": {"sync_merges": ctr["sync_merges"], "ack_resolved": ctr.get("ack_resolved_total", 0),
                           "diff_key_bytes": ctr["diff_key_bytes_total"], "ticks": ctr["tick"]},
            "exchange_ms_per_step": d["exchange_ns"] * 1e-6 / a.steps,
        }
        if a.workload not in ("c3",):  # the gossip plane dominates: whole-step algorithmic bytes against HBM
            line["metric"] = f"member·periods/sec, {a.workload.upper()} workload (not the headline)"
            line["roofline"] = {"bound": "hbm", "kernel": "whole step (k_gossip_send dominates)",
                                "achieved": B / dt / 1e9, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                                "frac": B / dt / 1e9 / HBM_PEAK_GBPS, "traffic": None}
            line["kernel_time_share"] = {}
        if a.rehearse_shard > 1:
            line["metric"] = "member·periods/sec of ONE slot shard, C5 rehearsal (not the headline)"
            line["config"]["parallelism"] = f"slot shard 0 of {a.rehearse_shard} (peers simulated)"
        if not a.no_cpu_baseline and world == 1:
            c.close()  # the engine's host buffers go before the oracle's tables
            c = None
            cm, cp = {"c3": (a.cpu_members, a.cpu_periods), "c3dyn": (a.cpu_members, a.cpu_periods),
                      "c2": (600, 40), "c5": (2000, 24)}[a.workload]
            if a.workload in ("c3", "c3dyn") and a.cpu_members is None:
                # the headline size when the host can hold the oracle's ~20 B per member pair (with 25 % slack),
                # 2 periods (~2 s each on 16 threads after ~1 min of setup); else 10k members, 120 periods
                cm, cp = (n, 2) if mem_available() > 25 * n * n else (10_000, 120)
            line["cpu_baseline"] = cpu_baseline(a, cm, cp)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if c is not None:
        c.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
