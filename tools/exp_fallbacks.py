"""Which exact fallbacks (include/swimhip_debug.h) a workload takes, per period: python tools/exp_fallbacks.py c2 [periods]
(SWIM_FALLBACKS=1 is set here; counts are cumulative since create)."""
import os
import sys
import time
from pathlib import Path

os.environ["SWIM_FALLBACKS"] = "1"
sys.path.insert(0, str(Path(__file__).resolve().parent.parent / "scalecube-cluster_amd"))
import swimhip  # noqa: E402
from swimhip import SimConfig, _abi  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "c2"
periods = int(sys.argv[2]) if len(sys.argv) > 2 else 14
n = 10_000 if w == "c2" else 100_000
c = swimhip.cluster(SimConfig(n_members=n))
if w == "c2":
    c.set_default_loss(5)
for p in range(1, periods + 1):
    if w == "c3dyn":
        c.update_incarnation((p * 7919) % n)
    t0 = time.time()
    c.run_periods(1)
    c.sync()
    fb = _abi.debug_fallbacks(c.lib, c._h)
    print(p, f"{(time.time() - t0) * 1e3:.1f} ms", {k: v for k, v in fb.items() if v}, flush=True)
c.close()
