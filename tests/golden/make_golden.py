"""Record the golden fixtures of tests/golden from the CPU oracle (oracle/swimref.cpp).

The reference (Java 8 + Reactor) cannot run in this image: there is no JDK. The oracle is its
restatement, pinned by the reference's own known-answer tests (tests/test_oracle_known_answers.py). These fixtures
freeze the oracle's behaviour on the C1 / C2 / C3 / C4 / C5 shapes so that any later change to either backend that moves a
single bit of state, a counter or an event shows up. Run from the repo root:  python tests/golden/make_golden.py [scenario ...]
"""
import json
import sys
import time
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
sys.path.insert(0, str(ROOT / "scalecube-cluster_amd"))
sys.path.insert(0, str(HERE))

from swimhip import _abi  # noqa: E402
from swimhip.cluster import SimulatedCluster  # noqa: E402

from scenarios import SCENARIOS, record  # noqa: E402


def main():
    lib = _abi.load(ROOT / "oracle" / "liboracle_swimref.so")
    only = set(sys.argv[1:])  # optional: scenario names to (re)record
    for name, make in SCENARIOS.items():
        if only and name not in only:
            continue
        cfg, _ = make()
        t0 = time.time()
        c = SimulatedCluster(lib, cfg)
        rec = record(c, name)
        c.close()
        rec["scenario"] = name
        rec["recorded_with"] = "oracle/swimref.cpp"
        (HERE / f"{name}.json").write_text(json.dumps(rec, separators=(",", ":")))
        print(name, len(rec["periods"]), "periods", "" if rec["events"] is None else f"{len(rec['events'])} events",
              f"{time.time() - t0:.1f} s")


if __name__ == "__main__":
    main()
