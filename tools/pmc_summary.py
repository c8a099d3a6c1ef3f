"""Summarise a tools/profile.sh output directory: per-kernel average duration
(kernel trace) and per-dispatch PMC counters, with the gfx950 FETCH_SIZE x2
correction (MI355X_MICROARCH.md §HBM).  Writes <dir>/summary.json."""
import collections
import csv
import json
import os
import sys

d = sys.argv[1]


def shorten(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0].split("::")[-1][:70]

out = {"kernels": {}, "pmc": {}}
ks = os.path.join(d, "trace", "run_kernel_stats.csv")
if os.path.exists(ks):
    for r in csv.DictReader(open(ks)):
        name = r["Name"]
        short = shorten(name)
        out["kernels"][short] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                                 "pct": float(r["Percentage"])}
for sub in sorted(os.listdir(d)):
    f = os.path.join(d, sub, "run_counter_collection.csv")
    if not sub.startswith("pmc") or not os.path.exists(f):
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        short = shorten(r["Kernel_Name"])
        agg[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in agg.items():
        out["pmc"].setdefault(k, {})[c] = sum(v) / len(v)
for k, c in out["pmc"].items():
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        # FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE reads half the bytes of wide streams
        c["hbm_bytes_est"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
    if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
        c["wait_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
json.dump(out, open(os.path.join(d, "summary.json"), "w"), indent=1)
for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["pct"])[:14]:
    print(f"{k[:60]:60s} calls={v['calls']:4d} avg={v['avg_us']:9.2f}us {v['pct']:5.1f}%")
for k, c in out["pmc"].items():
    print(k, {kk: (round(vv, 3) if vv < 1e3 else f"{vv:.3g}") for kk, vv in c.items()})
