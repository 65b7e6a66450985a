"""Debug: replay one golden scenario on the engine and report the first period that differs."""
import json
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scalecube-cluster_amd"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))
import swimhip
from swimhip.cluster import SimulatedCluster
from scenarios import SCENARIOS, record
name = sys.argv[1]
want = json.loads((ROOT / "tests" / "golden" / f"{name}.json").read_text())
cfg, _ = SCENARIOS[name]()
c = SimulatedCluster(swimhip.engine(), cfg)
rec = record(c, name)
for got, exp in zip(rec["periods"], want["periods"]):
    if got != exp:
        print("first diff at period", exp["period"], "got", got["counters"], "want", exp["counters"],
              "state", got["state"] == exp["state"], "events", got["events"] == exp["events"])
        break
else:
    print(name, "all periods equal")
