"""Per-kernel register / spill / occupancy table from hipcc's
-Rpass-analysis=kernel-resource-usage remarks (read on stdin).
Usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py [name-regex]"""
import re
import subprocess
import sys

pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"remark: (.*?) \[-Rpass-analysis", line)
    if not m:
        continue
    txt = m.group(1)
    if txt.startswith("Function Name:"):
        name = txt.split(":", 1)[1].strip()
        try:
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        except OSError:
            pass
        cur = {"name": name}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
keys = ["VGPRs", "AGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
for r in rows:
    if pat and not pat.search(r["name"]):
        continue
    nm = re.sub(r"^void ", "", r["name"]).replace("(anonymous namespace)::", "")
    nm = re.sub(r">\(.*", ">", nm)
    print(" | ".join(str(r.get(k, "-")) for k in keys), "|", nm[:110])
