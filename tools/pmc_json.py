"""gpurun_out/pmc_<tag>.json from the two PMC passes of tools/pmc_traffic.sh: the dominant kernel's HBM bytes per
dispatch, (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts half the bytes of wide streaming reads,
MI355X_MICROARCH.md §HBM).  The dominant kernel is the raster kernel dispatched most often in the run (the
fragment-counting variant runs once)."""
import collections
import csv
import glob
import json
import os
import statistics
import sys

d, tag, args = sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else ""
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(d, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
cand = [(len(v.get("FETCH_SIZE", [])), k) for k, v in vals.items() if v.get("FETCH_SIZE") and v.get("WRITE_SIZE")]
n, k = max(cand)
# per-dispatch median: a few dispatches of a gated batch (k_gate_wait polling beside it) read absurd FETCH_SIZE
# values under --pmc's serialised dispatch (12 GB in a 30 us kernel, round 5), so the mean is not used
fetch = statistics.median(vals[k]["FETCH_SIZE"])
write = statistics.median(vals[k]["WRITE_SIZE"])
out = {"kernel": k.replace("void ", "").replace("nrtri::(anonymous namespace)::", "").split("(")[0], "config": tag,
       "bench_args": args, "hbm_bytes_per_launch": int((2 * fetch + write) * 1024),
       "FETCH_SIZE_KiB": fetch, "WRITE_SIZE_KiB": write, "dispatches": n,
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (bench.py --steps 3 --warmup 1), "
                 "per-dispatch median; bytes = (2*FETCH_SIZE + WRITE_SIZE)*1024 (gfx950 FETCH_SIZE halving)"}
json.dump(out, open(os.path.join(os.path.dirname(d), f"pmc_{tag}.json"), "w"), indent=1)
print(json.dumps(out))
