"""Per-tick kernel time breakdown from a rocprofv3 kernel trace (run_kernel_trace.csv): each tick starts at a
k_member_tick dispatch; prints the last `n` ticks' per-kernel durations (us) and the tick's span."""
import collections
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ticks, cur = [], None
for r in rows:
    name = r["Kernel_Name"].split("(")[0].replace("swim::", "").replace("void ", "")
    if name.startswith("k_member_tick") and not name.endswith("<2u>"):  # <2u>: the resume launch of a split tick
        cur = collections.OrderedDict(_start=int(r["Start_Timestamp"]))
        ticks.append(cur)
    if cur is None:
        continue
    cur[name] = cur.get(name, 0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cur["_end"] = int(r["End_Timestamp"])
tot = collections.Counter()
for t in ticks[-n:]:
    busy = sum(v for k, v in t.items() if not k.startswith("_"))
    span = (t["_end"] - t["_start"]) / 1e3
    top = sorted(((v, k) for k, v in t.items() if not k.startswith("_")), reverse=True)[:6]
    print(f"span {span:8.1f} us busy {busy:8.1f}: " + ", ".join(f"{k} {v:.0f}" for v, k in top))
    for k, v in t.items():
        if not k.startswith("_"):
            tot[k] += v
nt = min(n, len(ticks))
spans = [(t["_end"] - t["_start"]) / 1e3 for t in ticks[-n:]]
print("mean over the last", nt, "ticks:", ", ".join(f"{k} {v / nt:.0f}" for k, v in tot.most_common(10)))
if len(sys.argv) > 3:  # every kernel, and the mean span / busy time
    print(f"mean span {sum(spans) / nt:.1f} us, busy {sum(tot.values()) / nt:.1f} us")
    for k, v in tot.most_common():
        print(f"  {k:40s} {v / nt:8.1f}")
