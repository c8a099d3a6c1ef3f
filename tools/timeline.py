"""Kernel timeline of the last frames of a rocprofv3 --kernel-trace CSV:
start/end (us, relative) and the gap before each dispatch, so overlaps and
bubbles between the binning stream and the raster stream can be read.
Usage: python tools/timeline.py <kernel_trace.csv> [frames=3] [anchor=k_vis]"""
import csv
import re
import sys

path = sys.argv[1]
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 3
anchor = sys.argv[3] if len(sys.argv) > 3 else "k_vis"
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        name = r.get("Kernel_Name") or r.get("KernelName") or ""
        s = int(r.get("Start_Timestamp") or r.get("BeginNs"))
        e = int(r.get("End_Timestamp") or r.get("EndNs"))
        q = r.get("Queue_Id") or r.get("Stream_Id") or r.get("queue-id") or "?"
        short = name.replace("(anonymous namespace)::", "").replace("nrtri::", "")
        short = re.sub(r"\(.*", "", re.sub(r"^void ", "", short))
        rows.append((s, e, short[:48], q))
rows.sort()
idx = [i for i, r in enumerate(rows) if anchor in r[2]]
if len(idx) < frames + 1:
    sys.exit("not enough anchor kernels")
first = idx[-frames - 1]
t0 = rows[first][0]
prev_end = {}
print(f"{'start':>9} {'end':>9} {'dur':>7} {'gap':>7}  queue  kernel")
for s, e, n, q in rows[first:]:
    gap = (s - prev_end[q]) / 1e3 if q in prev_end else float('nan')
    prev_end[q] = e
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {gap:7.1f}  {q:>5}  {n}")
ks = [rows[i] for i in idx[-frames - 1:]]
per = [(ks[i + 1][0] - ks[i][0]) / 1e3 for i in range(len(ks) - 1)]
print("anchor period (us):", " ".join(f"{p:.1f}" for p in per))

# optional: HIP runtime API calls (rocprofv3 --hip-runtime-trace) in the same window
import glob
import os
api = glob.glob(os.path.join(os.path.dirname(path), "*hip_api_trace.csv"))
if api:
    t_end = rows[-1][1]
    calls = []
    with open(api[0]) as f:
        for r in csv.DictReader(f):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s >= t0 and s <= t_end:
                calls.append((s, e, r["Function"]))
    calls.sort()
    print("\nHIP API calls in the window (start, dur us):")
    for s, e, fn in calls:
        if fn in ("hipGetLastError", "hipGetDevice", "hipSetDevice"):
            continue
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {fn}")
