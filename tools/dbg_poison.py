"""Debug: which allocation's initial contents change the result? Poison one allocation at a time."""
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scalecube-cluster_amd"))
import swimhip  # noqa: E402
from swimhip import SimConfig, _abi  # noqa: E402
from swimhip.cluster import SimulatedCluster  # noqa: E402

ora = _abi.load(ROOT / "oracle" / "liboracle_swimref.so")
eng = swimhip.engine()
cfg = SimConfig(n_members=300, record_events=True)
o = SimulatedCluster(ora, cfg)
o.set_default_loss(5)
o.step(30)
ref = o.state_hash()
bad = []
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 130):
    os.environ["SWIM_POISON_ONLY"] = str(i)
    e = SimulatedCluster(eng, cfg)
    e.set_default_loss(5)
    e.step(30)
    h = e.state_hash()
    if not np.array_equal(h, ref):
        d = np.argwhere(h != ref)
        bad.append(i)
        print(f"alloc #{i}: differs ({len(d)} words, first member {d[0][0]} word {d[0][1]})", flush=True)
    e.close()
os.environ.pop("SWIM_POISON_ONLY")
print("culprits:", bad, flush=True)
