"""C4-shaped: N members PRECONVERGED, two halves blocked both ways from period 0, unblockAll at period
`heal`, run to period `end`; prints wall time per 20-period chunk and the counters (gossip created, events)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scalecube-cluster_amd"))
import os  # noqa: E402

# the DEAD-gossip storm delivers ~10^8 first receipts a tick; the engine grows its slot table, receipt rings and
# per-tick receipt lists as the storm builds (api.hip grow_caps), so no capacity is set here unless asked for
import swimhip  # noqa: E402
from swimhip import ClusterConfig, SimConfig  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
heal = int(sys.argv[2]) if len(sys.argv) > 2 else 200
end = int(sys.argv[3]) if len(sys.argv) > 3 else 320
slots = int(sys.argv[4]) if len(sys.argv) > 4 else 0  # 0: the engine's default (grown as needed)
ring = int(os.environ.get("C4_RING", "0"))  # receipt-ring entries per member (0: the engine's default)
c = swimhip.cluster(SimConfig(n_members=n, cluster=ClusterConfig(seedMembers=[0]), gossip_slot_cap=slots,
                              pending_fetch_cap=16384, list_slack=4096,  # the heal re-adds a whole side at once
                              gossip_ring_cap=ring))
print(f"N={n}: device bytes {c.counters()['device_bytes'] / 2**30:.1f} GiB", flush=True)
c.partition([0] * (n // 2) + [1] * (n - n // 2))
p, t_all = 0, time.perf_counter()
while p < end:
    if p == heal:
        c.unblock_all()
    step = min(int(os.environ.get("C4_CHUNK", "10")), (heal if p < heal else end) - p)
    t0 = time.perf_counter()
    try:
        c.run_periods(step)
        c.sync()
    except Exception as x:  # capacity / memory: report how far it got
        print(f"N={n} stopped in periods {p}-{p + step}: {x}; device bytes "
              f"{c.counters()['device_bytes'] / 2**30:.1f} GiB", flush=True)
        raise SystemExit(2)
    dt = time.perf_counter() - t0
    p += step
    ctr = c.counters()
    print(f"N={n} periods {p - step}-{p}: {dt / step * 1e3:.1f} ms/period, created {ctr['gossips_created']}, "
          f"events {ctr['events']}, G {ctr['gossip_messages']}, device {ctr['device_bytes'] / 2**30:.1f} GiB",
          flush=True)
    if os.environ.get("C4_SUSPECT"):  # sampled observers: how much of the other side each one holds SUSPECT
        import numpy as np
        half = n // 2
        obs = list(range(0, half, max(1, half // 16))) + list(range(half, n, max(1, half // 16)))
        fr = []
        for o in obs:
            st = (c.row(o) >> np.uint64(32)) & np.uint64(3)
            other = st[half:] if o < half else st[:half]
            own = st[:half] if o < half else st[half:]
            fr.append(((other == 2).mean(), (own == 1).mean()))  # SUSPECT on the other side, ALIVE on its own
        fr = np.array(fr)
        print(f"   SUSPECT share of the other side: min {fr[:, 0].min():.4f} mean {fr[:, 0].mean():.4f}; "
              f"own side ALIVE min {fr[:, 1].min():.4f}", flush=True)
print(f"N={n} total {time.perf_counter() - t_all:.1f} s for {end} periods", flush=True)
c.close()
