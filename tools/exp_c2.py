import sys, time
sys.path.insert(0, "scalecube-cluster_amd")
import swimhip
from swimhip import SimConfig
N = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
c = swimhip.cluster(SimConfig(n_members=N, profile=True))
c.set_default_loss(5)
t = time.perf_counter(); c.run_periods(10); print("warm 10 periods", time.perf_counter() - t, c.counters(), flush=True)
for r in range(3):
    b = c.counters(); t = time.perf_counter(); c.run_periods(10); dt = time.perf_counter() - t; e = c.counters()
    d = {k: e[k] - b[k] for k in e}
    print(f"10 periods: {dt:.3f}s -> {N*10/dt:.3e} member-periods/s; member {d['member_ns']/1e6:.1f} ms diff {d['diff_ns']/1e6:.1f} ms gossip_send {d['gossip_ns']/1e6:.1f} ms; G={d['gossip_messages']:.3e} E={d['events']} created={d['gossips_created']}", flush=True)
