"""Summary of a GPU session's bench lines (gpurun_out/<tag>/*.log): per log,
the environment / step name, ms per step and the per-kernel microseconds.
Usage: python tools/ab_summary.py gpurun_out/<tag>"""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.log"))):
    for line in open(f, errors="replace"):
        if line.startswith("{") and '"ms_per_step"' in line:
            d = json.loads(line)
            ks = " ".join(f"{k}={v}" for k, v in d.get("kernel_us", {}).items())
            r = d.get("roofline", {})
            print(f"{os.path.basename(f)[:60]:60s} {d['ms_per_step']:.4f} ms  frac={r.get('frac')} "
                  f"path_frac={r.get('path_frac')}  {ks}")
