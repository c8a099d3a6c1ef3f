"""Steady-state kernel times from a rocprofv3 kernel trace of bench.py.

rocprofv3 --stats averages every dispatch of the run.  bench.py's clock-settle
phase renders frames in groups of four with a drain after each group, so there
the next frame's binning does not run beside the raster, and the raster is
~10 % faster than in the steady state that the kernel pass and the timed region
measure (binning beside the raster, profiles/r06/README.md).  This prints, per
kernel, the average over all dispatches and over the last N dispatches (the
kernel pass + timed region + verification frames of a --steps K run: N = 2K +
a few).

    python tools/trace_steady.py run_kernel_trace.csv [N] [name-regex]
"""
import csv
import re
import statistics
import sys


def main():
    path = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    rx = re.compile(sys.argv[3] if len(sys.argv) > 3 else "k_vis|k_tile_raster|k_bin_warm|k_free")
    by = {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not rx.search(name):
            continue
        short = name.replace("void ", "").replace("nrtri::(anonymous namespace)::", "").split("(")[0]
        by.setdefault(short, []).append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    print(f"{'kernel':48s} {'calls':>6s} {'avg us':>8s} {'last-N avg':>11s} {'last-N median':>14s}  (N = {n})")
    for k, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
        v.sort()
        d = [x[1] for x in v]
        last = d[-n:]
        print(f"{k:48s} {len(d):6d} {statistics.mean(d):8.2f} {statistics.mean(last):11.2f} {statistics.median(last):14.2f}")


if __name__ == "__main__":
    main()
