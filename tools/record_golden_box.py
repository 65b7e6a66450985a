"""Record a golden fixture from the CPU oracle on the GPU box (its host RAM and cores), period by period.

The box-sized scenarios (tests/golden/scenarios.py BOX_SCENARIOS: C3 at 100 000 members, C2 at 10 000 past period 3, C4
at 50 000) need more host RAM than this container's 64 GB. The oracle runs there on SWIMREF_THREADS workers (no GPU is
used); the record is rewritten after every period, so a run stopped by its memory guard keeps every finished period.

  python3 tools/record_golden_box.py NAME [--max-periods P] [--mem-gb G] [--out DIR]

A heartbeat line every 30 s (elapsed, RSS) keeps gpurun's hang detector quiet through long periods. When the RSS passes
--mem-gb the process exits with status 3 (the periods finished so far are on disk), before the box's memory cap.
"""
import argparse
import json
import os
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scalecube-cluster_amd"))
sys.path.insert(0, str(ROOT / "tests" / "golden"))

from swimhip import _abi  # noqa: E402
from swimhip.cluster import SimulatedCluster  # noqa: E402

from scenarios import BOX_SCENARIOS, SCENARIOS, record  # noqa: E402


def rss():
    for line in open("/proc/self/status"):
        if line.startswith("VmRSS:"):
            return int(line.split()[1]) * 1024
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--max-periods", type=int, default=None)
    ap.add_argument("--mem-gb", type=float, default=245.0)
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "golden"))
    a = ap.parse_args()
    os.environ.setdefault("SWIMREF_THREADS", "16")
    out_dir = Path(a.out)
    out_dir.mkdir(parents=True, exist_ok=True)
    dst = out_dir / f"{a.name}.json"
    t0 = time.time()
    peak = [0]
    state = {"period": 0, "t_period": t0}

    def guard():
        last = 0.0
        while True:
            time.sleep(1.0)
            r = rss()
            peak[0] = max(peak[0], r)
            if r > a.mem_gb * 1e9:
                print(f"MEMORY GUARD: RSS {r / 1e9:.1f} GB > {a.mem_gb} GB in period {state['period'] + 1}; "
                      f"{state['period']} periods recorded in {dst}", flush=True)
                os._exit(3)
            if time.time() - last >= 30:
                last = time.time()
                print(f"  ... {time.time() - t0:.0f} s, period {state['period'] + 1} running "
                      f"{time.time() - state['t_period']:.0f} s, RSS {r / 1e9:.1f} GB", flush=True)

    threading.Thread(target=guard, daemon=True).start()
    lib = _abi.load(ROOT / "oracle" / "liboracle_swimref.so")
    cfg, _ = {**SCENARIOS, **BOX_SCENARIOS}[a.name]()
    c = SimulatedCluster(lib, cfg)
    print(f"{a.name}: {cfg.n_members} members, oracle on {os.environ['SWIMREF_THREADS']} threads, set up in "
          f"{time.time() - t0:.1f} s, RSS {rss() / 1e9:.1f} GB", flush=True)

    def on_period(rec):
        p = len(rec["periods"])
        now = time.time()
        body = dict(rec, scenario=a.name, recorded_with="oracle/swimref.cpp",
                    recorded_on=f"GPU box host, SWIMREF_THREADS={os.environ['SWIMREF_THREADS']}",
                    period_seconds=round(now - state["t_period"], 2), peak_rss_gb=round(peak[0] / 1e9, 1))
        tmp = dst.with_suffix(".tmp")
        tmp.write_text(json.dumps(body, separators=(",", ":")))
        tmp.replace(dst)
        ctr = rec["periods"][-1]["counters"]
        print(f"{a.name} period {p}: {now - state['t_period']:.1f} s, RSS {rss() / 1e9:.1f} GB (peak "
              f"{peak[0] / 1e9:.1f}), counters {ctr}", flush=True)
        state["period"] = p
        state["t_period"] = now

    record(c, a.name, limit=a.max_periods, on_period=on_period)
    print(f"{a.name}: done, {state['period']} periods in {time.time() - t0:.0f} s, peak RSS {peak[0] / 1e9:.1f} GB",
          flush=True)
    os._exit(0)  # skip the oracle's teardown of ~10^10 table entries


if __name__ == "__main__":
    main()
