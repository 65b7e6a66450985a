"""Per-tick HBM bytes and L2 atomics of the gossip data plane from three rocprofv3 --pmc passes (FETCH_SIZE with the
gfx950 x2 correction, WRITE_SIZE, TCC_ATOMIC_sum; MI355X_MICROARCH.md HBM section), averaged over the last <timed ticks>
member-kernel dispatches (= ticks) and the dispatches after the first of them. Usage: python tools/pmc_gossip.py <dir> <workload> <timed ticks> [out.json]
<dir> holds pmc_<workload>_<counter>/run_counter_collection.csv (tools/gpu_run.sh step pmcg), exp4_<workload>.log and
t_<workload>/run_kernel_stats.csv. A tick starts at each k_member_tick dispatch that is not the resume launch of a split
tick (k_member_tick_t<2u>)."""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, last):
    """counter sums per kernel over the dispatches of the last `last` ticks (the timed periods of the bench run)"""
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        full = r["Kernel_Name"].split("(")[0].replace("swim::", "").replace("void ", "")
        r["name"] = full.split("<")[0]
        r["tick"] = full.startswith("k_member_tick") and not full.endswith("<2u>")
    ticks = sorted({int(r["Dispatch_Id"]) for r in rows if r["tick"]})
    first = ticks[-last] if last and len(ticks) >= last else 0
    tot, disp = defaultdict(float), defaultdict(set)
    for r in rows:
        if int(r["Dispatch_Id"]) < first:
            continue
        tot[r["name"]] += float(r["Counter_Value"])
        disp[r["name"]].add(r["Dispatch_Id"])
    nd = {k: len(v) for k, v in disp.items()}
    nd["_ticks"] = len([t for t in ticks if t >= first])
    return tot, nd


def main():
    d, w, last = sys.argv[1], sys.argv[2], int(sys.argv[3])
    f, nd = per_kernel(f"{d}/pmc_{w}_FETCH_SIZE/run_counter_collection.csv", last)
    wr, _ = per_kernel(f"{d}/pmc_{w}_WRITE_SIZE/run_counter_collection.csv", last)
    try:
        at, _ = per_kernel(f"{d}/pmc_{w}_TCC_ATOMIC_sum/run_counter_collection.csv", last)
    except FileNotFoundError:
        at = {}
    ticks = max(1, nd.pop("_ticks"))
    out = {"ticks": ticks, "kernels": {}}
    for k in sorted(f, key=lambda k: -(2 * f[k] + wr.get(k, 0))):
        out["kernels"][k] = {"dispatches": nd[k], "hbm_bytes_per_tick": (2 * f[k] + wr.get(k, 0)) * 1024 / ticks,
                             "fetch_bytes_per_tick_x2": 2 * f[k] * 1024 / ticks,
                             "write_bytes_per_tick": wr.get(k, 0) * 1024 / ticks,
                             "l2_atomics_per_tick": at.get(k, 0) / ticks}
    gk = [k for k in out["kernels"] if not k.startswith("k_member_tick") and k != "k_inbox_apply"]
    out["gossip_plane_hbm_bytes_per_tick"] = sum(out["kernels"][k]["hbm_bytes_per_tick"] for k in gk)
    out["gossip_plane_l2_atomics_per_tick"] = sum(out["kernels"][k]["l2_atomics_per_tick"] for k in gk)
    # the same ticks' op counters from the bench line of the FETCH_SIZE pass: SURVEY.md §8d algorithmic bytes
    # B = 8R + 8W + 32M + 0.375G + 24E (4-B record keys) against the measured HBM bytes of the whole step
    line = [json.loads(x) for x in open(f"{d}/pmc_{w}_FETCH_SIZE.log") if x.startswith("{")]
    if line:
        c, ticks = line[-1]["counters"], line[-1]["steps"] * line[-1]["config"]["ticks_per_period"]
        B = 8 * c["record_compares"] + 8 * c["row_writes"] + 32 * c["messages"] + 0.375 * c["gossip_messages"] + 24 * c["events"]
        out["algorithmic_bytes_per_tick"] = B / ticks
        out["counters_per_tick"] = {k: v / ticks for k, v in c.items()}
        allb = sum(v["hbm_bytes_per_tick"] for v in out["kernels"].values())
        out["hbm_bytes_per_tick_all_kernels"] = allb
        out["wasted_traffic_ratio"] = allb / (B / ticks) if B else None
    # k_gossip_send's algorithmic bytes from the same ticks' work units (SWIM_EXP=4 run of the same command, the
    # workload is deterministic): an 8-B held word per (target, active group) item, an 8-B window word per sender of
    # the item, a 4-B ring entry per first-receipt candidate. Atomic throughput from the kernel-trace averages.
    try:
        ex = [x for x in open(f"{d}/exp4_{w}.log") if x.startswith("exp: items")][-(last // 10 or 1):]
        tok = lambda x, key: int(x.split(key)[1].split()[0])
        n = len(ex) * 10  # one line per step (one period = 10 ticks)
        items, words = sum(tok(x, "target-group items ") for x in ex) / n, sum(tok(x, "sender words ") for x in ex) / n
        cand = sum(tok(x, "candidates ") for x in ex) / n
        alg = 8 * items + 8 * words + 4 * cand
        ks = out["kernels"].get("k_gossip_send")
        if ks:
            ks["algorithmic_bytes_per_tick"] = alg
            ks["traffic_ratio"] = ks["hbm_bytes_per_tick"] / alg if alg else None
            ks["work_units_per_tick"] = {"target_group_items": items, "sender_words": words, "candidates": cand}
    except FileNotFoundError:
        pass
    try:
        for r in csv.DictReader(open(f"{d}/t_{w}/run_kernel_stats.csv")):
            k = r["Name"].split("(")[0].replace("swim::", "").replace("void ", "").split("<")[0]
            if k in out["kernels"]:
                us = float(r["AverageNs"]) / 1e3
                e = out["kernels"][k]
                e["avg_us"] = us
                e["achieved_GBps"] = e["hbm_bytes_per_tick"] / max(1, e["dispatches"] / ticks) / us / 1e3
                e["l2_atomics_per_us"] = e["l2_atomics_per_tick"] / max(1, e["dispatches"] / ticks) / us
    except FileNotFoundError:
        pass
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 4:
        json.dump(out, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
