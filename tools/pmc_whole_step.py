"""Whole-step HBM bytes per period from rocprofv3 PMC passes (tools/gpu_run.sh pmc:W:FETCH_SIZE:S and WRITE_SIZE:S).

Two bench runs of different lengths (S1 < S2 timed periods, same warm-up) per counter: the difference of their totals
over every kernel dispatch is the traffic of S2 - S1 steady periods, free of the one-off initialisation kernels.
FETCH_SIZE / WRITE_SIZE are KB per dispatch; FETCH_SIZE is doubled (gfx950 tallies wide coalesced reads at half,
MI355X_MICROARCH.md HBM / rocprofv3 section). Writes / updates profiles/pmc_whole_step.json[workload] and copies the
counter CSVs into profiles/ as <round>_pmc_whole_<workload>_<counter>_<S>.csv.

  python tools/pmc_whole_step.py <gpurun_out dir> <workload> <members> <round tag> <S1> <S2>
"""
import collections
import csv
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def totals(d):
    f = next(d.rglob("*counter_collection.csv"))
    per = collections.Counter()
    for r in csv.DictReader(open(f)):
        per[r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()] += float(r["Counter_Value"]) * 1024
    return per, f


def main():
    src, w, n, tag, s1, s2 = Path(sys.argv[1]), sys.argv[2], int(sys.argv[3]), sys.argv[4], int(sys.argv[5]), int(sys.argv[6])
    prof = ROOT / "profiles"
    out = {}
    for ctr, mult in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
        (a, fa), (b, fb) = totals(src / f"pmc_{w}_{ctr}_{s1}"), totals(src / f"pmc_{w}_{ctr}_{s2}")
        diff = {k: mult * (b[k] - a.get(k, 0.0)) / (s2 - s1) for k in b}
        out[ctr] = diff
        for s, f in ((s1, fa), (s2, fb)):
            shutil.copy(f, prof / f"{tag}_pmc_whole_{w}_{ctr}_{s}.csv")
    kernels = sorted(set(out["FETCH_SIZE"]) | set(out["WRITE_SIZE"]),
                     key=lambda k: -(out["FETCH_SIZE"].get(k, 0) + out["WRITE_SIZE"].get(k, 0)))
    per_kernel = {k: round(out["FETCH_SIZE"].get(k, 0) + out["WRITE_SIZE"].get(k, 0)) for k in kernels[:12]}
    rec = {"round": tag, "members": n, "periods": s2 - s1,
           "bytes_per_period": sum(out["FETCH_SIZE"].values()) + sum(out["WRITE_SIZE"].values()),
           "fetch_bytes_per_period_x2": sum(out["FETCH_SIZE"].values()),
           "write_bytes_per_period": sum(out["WRITE_SIZE"].values()),
           "top_kernels_bytes_per_period": per_kernel,
           "method": f"bench.py --workload {w}: ({s2}-step run - {s1}-step run) / {s2 - s1}, FETCH_SIZE x2 + WRITE_SIZE"}
    f = prof / "pmc_whole_step.json"
    allrec = json.loads(f.read_text()) if f.exists() else {}
    allrec[w] = rec
    f.write_text(json.dumps(allrec, indent=1))
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
