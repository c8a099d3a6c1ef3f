"""Parses hipcc -Rpass-analysis=kernel-resource-usage remarks (stdin) into one
line per kernel instance: VGPRs, AGPRs, scratch bytes per lane, occupancy,
LDS bytes.  Usage: ... | python tools/kres_parse.py [name-regex]"""
import re
import subprocess
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "."
cur, rows = None, []
keys = (("vgpr", r" VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
        ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)"))
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key, p in keys:
        m = re.search(p, line)
        if m and cur is not None:
            cur[key] = m.group(1)
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True, text=True).stdout.split("\n")
for r, n in zip(rows, names):
    n = re.sub(r"\(.*", "", n.replace("nrtri::(anonymous namespace)::", ""))
    if re.search(pat, n):
        print("%-52s vgpr=%s agpr=%s scratch=%s occ=%s lds=%s" % (n, r.get("vgpr"), r.get("agpr"), r.get("scratch"),
                                                                   r.get("occ"), r.get("lds")))
