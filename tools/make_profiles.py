"""Copy a round's GPU profile outputs into profiles/ and summarise the k_sync_diff PMC passes.

FETCH_SIZE / WRITE_SIZE are in KB per dispatch; on gfx950 FETCH_SIZE counts wide coalesced streaming reads at half
(MI355X_MICROARCH.md, HBM / rocprofv3 section), so it is doubled. Launches of the first two ticks (empty message
lists) are dropped; the median of the rest is the steady-state traffic per launch."""
import csv
import json
import shutil
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
src = ROOT / "gpurun_out" / "round"
tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
prof = ROOT / "profiles"


def values(path):
    rows = list(csv.DictReader(open(path)))
    return [float(r["Counter_Value"]) for r in rows if "k_sync_diff" in r["Kernel_Name"]]


def pass_totals(d):
    """the bench line of a PMC pass: its run_totals price the same launches the pass counted"""
    for line in (src / f"{d}.log").read_text().splitlines():
        if line.startswith("{") and "run_totals" in line:
            return json.loads(line)["run_totals"]
    return None


fetch_all = values(next((src / "pmc_fetch").rglob("*counter_collection.csv")))
write_all = values(next((src / "pmc_write").rglob("*counter_collection.csv")))
fetch = [x for x in fetch_all if x > 1000.0]  # steady-state launches (the first ticks carry no SYNC payloads)
write = [x for x in write_all if x > 1000.0]
stats = next((src / "trace").rglob("*kernel_stats.csv"))
avg_us = None
for r in csv.DictReader(open(stats)):
    if "k_sync_diff" in r["Name"]:
        avg_us = float(r["AverageNs"]) / 1e3
bench = json.loads((src / "bench.json").read_text())
n = bench["config"]["members"]
fm, wm = statistics.median(fetch), statistics.median(write)
# like-for-like: every k_sync_diff launch of the two PMC passes against the algorithmic bytes of those same launches
# (the key bytes the engine counted over each pass's whole run, warm-up included: 2 B x N per payload streamed from
# the 8-bit shadow plane, 8 B x N per other payload)
tf, tw = pass_totals("pmc_fetch"), pass_totals("pmc_write")
ratio = None
if tf and tw:
    measured = 2 * sum(fetch_all) * 1024 + sum(write_all) * 1024  # one FETCH pass + one WRITE pass (same schedule)
    # (SYNC_ACKs resolved from write logs are merged without being streamed: k_ack_resolve)
    streamed = lambda t: t["sync_merges"] - t.get("ack_resolved", 0)
    kb = lambda t: t["diff_key_bytes"] if "diff_key_bytes" in t else 8.0 * n * streamed(t)
    algo = (kb(tf) + kb(tw)) / 2
    ratio = measured / algo
out = {
    "round": int(tag[1:]),
    "members": n,
    "kernel": "k_sync_diff",
    "workload": "C3 steady state, bench.py --steps 3 --warmup 1 (8-bit shadow key plane)",
    "fetch_size_kb_median": fm,
    "write_size_kb_median": wm,
    "gfx950_fetch_correction": "FETCH_SIZE x2 (MI355X_MICROARCH.md HBM section: wide coalesced reads are tallied at half)",
    "bytes_per_launch": 2 * fm * 1024 + wm * 1024,
    "algorithmic_bytes_per_launch": bench["roofline"]["algorithmic_bytes_per_launch"],
    "traffic_over_algorithmic_same_launches": ratio,
    "rocprof_avg_duration_us": avg_us,
    "bench_hip_event_avg_us": bench["roofline"]["avg_launch_us"],
    "source_files": [f"{tag}_pmc_fetch_size_sync_diff.csv", f"{tag}_pmc_write_size_sync_diff.csv",
                     f"{tag}_kernel_stats_c3_100k.csv"],
}
(prof / "pmc_sync_diff_k8.json").write_text(json.dumps(out, indent=1))
shutil.copy(next((src / "pmc_fetch").rglob("*counter_collection.csv")), prof / f"{tag}_pmc_fetch_size_sync_diff.csv")
shutil.copy(next((src / "pmc_write").rglob("*counter_collection.csv")), prof / f"{tag}_pmc_write_size_sync_diff.csv")
shutil.copy(stats, prof / f"{tag}_kernel_stats_c3_100k.csv")
(prof / f"{tag}_bench_c3_100k.json").write_text((src / "bench.json").read_text())
print(json.dumps(out, indent=1))
