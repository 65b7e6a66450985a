"""One-off CPU baseline at the headline size: the oracle (oracle/swimref.cpp, a port) on C3 at 100k members, all host
worker threads (at most 16), 1 warm-up period then 2 timed periods; writes a JSON record (bench.py's cpu_baseline shape).
Needs ~200 GB of host RAM (20 B per member pair) and a few minutes of setup; the default bench samples 10k instead."""
import json
import os
import resource
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scalecube-cluster_amd"))
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
periods = int(sys.argv[2]) if len(sys.argv) > 2 else 2
out = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/cpu_baseline_full.json"
cores = max(1, min(16, len(os.sched_getaffinity(0))))
os.environ["SWIMREF_THREADS"] = str(cores)
from swimhip import SimConfig, _abi  # noqa: E402
from swimhip.cluster import SimulatedCluster  # noqa: E402

lib = _abi.load(ROOT / "oracle" / "liboracle_swimref.so")
t0 = time.perf_counter()
c = SimulatedCluster(lib, SimConfig(n_members=n))
t1 = time.perf_counter()
print(f"setup {t1 - t0:.1f} s", flush=True)
c.run_periods(1)
t2 = time.perf_counter()
print(f"warm-up period {t2 - t1:.1f} s", flush=True)
c.run_periods(periods)
dt = time.perf_counter() - t2
rec = {"value": n * periods / dt, "unit": "member·periods/s", "cores": cores, "kind": "port",
       "sample": f"oracle/swimref.cpp on C3 at {n} members (the headline size), {periods} periods after 1 warm-up "
                 f"period on {cores} worker threads: {dt:.1f} s timed, setup {t1 - t0:.1f} s",
       "max_rss_gb": resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1e6,
       "counters": c.counters()}
c.close()
Path(out).write_text(json.dumps(rec, indent=1))
print(json.dumps(rec), flush=True)
