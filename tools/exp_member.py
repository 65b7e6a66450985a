import sys, time
sys.path.insert(0, "scalecube-cluster_amd")
import swimhip
from swimhip import SimConfig, ClusterConfig
N = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
for name, cc in [("default", ClusterConfig()), ("nosync", ClusterConfig(syncInterval=3_000_000)),
                 ("noping", ClusterConfig(pingInterval=1_000_000)), ("neither", ClusterConfig(syncInterval=3_000_000, pingInterval=1_000_000))]:
    c = swimhip.cluster(SimConfig(n_members=N, cluster=cc, profile=True))
    c.step(20)
    b = c.counters(); t = time.perf_counter(); c.step(100); dt = time.perf_counter() - t; e = c.counters()
    print(f"{name:8s} member_us/tick={(e['member_ns']-b['member_ns'])/100/1e3:8.1f} diff_us/tick={(e['diff_ns']-b['diff_ns'])/100/1e3:8.1f} wall_us/tick={dt*1e4:8.1f}", flush=True)
    c.close()
