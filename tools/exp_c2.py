"""C2: N members (default 10k), PRECONVERGED, 5 % loss on every link, one GPU.
Prints the per-period gossip load (created, sends G, events E) and the throughput after warm-up."""
import sys, time
sys.path.insert(0, "scalecube-cluster_amd")
import swimhip
from swimhip import SimConfig
N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
P = int(sys.argv[2]) if len(sys.argv) > 2 else 30
c = swimhip.cluster(SimConfig(n_members=N, profile=True))
c.set_default_loss(5)
prev = c.counters()
t0 = time.perf_counter()
tw = None
for p in range(P):
    t = time.perf_counter()
    c.run_periods(1)
    c.sync()
    dt = time.perf_counter() - t
    e = c.counters()
    d = {k: e[k] - prev[k] for k in e}
    prev = e
    print(f"period {p}: {dt*1e3:.1f} ms created {d['gossips_created']} G {d['gossip_messages']:.3e} E {d['events']} "
          f"R {d['record_compares']:.3e} member {d['member_ns']/1e6:.1f} ms diff {10 * d['diff_ns'] / max(1, d['diff_launches']) / 1e6:.1f} ms", flush=True)  # every 5th tick's diff is timed
    if p == 9:
        tw = time.perf_counter()
if tw is not None and P > 10:
    dt = time.perf_counter() - tw
    print(f"C2 steady state (periods 10..{P-1}): {dt/(P-10)*1e3:.1f} ms/period -> {N*(P-10)/dt:.3e} member-periods/s", flush=True)
