"""A/B variant source patch: the plan kernels' host totals as 64-bit words (seq << 32) | value, each stored on
its own without a system-scope release (which writes back the whole L2: buffer_wbl2 sc0 sc1), the host
waiting until every word carries the batch's sequence number.  Usage: python patch_nowb.py <csrc dir>"""
import re
import sys

d = sys.argv[1]
p = d + "/nr_common.h"
s = open(p).read()
s = s.replace("        u32* h_plan = nullptr;", "        u64* h_plan = nullptr;").replace("        u32* d_hplan = nullptr;", "        u64* d_hplan = nullptr;")
assert "u64* h_plan" in s and "u64* d_hplan" in s
open(p, "w").write(s)
p = d + "/nr_tri_free.hip"
s = open(p).read()
s = s.replace("u32* __restrict__ host_totals", "u64* __restrict__ host_totals")
pat = re.compile(r"(?P<ind>[ ]*)const u32 t\[4\] = \{ta, tb, tm, fits \? 1u : 0u\};\n.*?"
                 r"__hip_atomic_store\(&host_totals\[4\], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM\);\n", re.S)


def rep(m):
    ind = m.group("ind")
    return (f"{ind}const u32 t[6] = {{ta, tb, tm, fits ? 1u : 0u, seq, th}};\n"
            f"{ind}for (int k = 0; k < 4; ++k) totals[k] = t[k];\n"
            f"{ind}for (int k = 0; k < 6; ++k)\n"
            f"{ind}    __hip_atomic_store(&host_totals[k], ((u64)seq << 32) | t[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);\n")


s, n = pat.subn(rep, s)
assert n == 3, n
s = s.replace("8 * sizeof(u32), hipHostMallocMapped | hipHostMallocCoherent));\n        F.h_plan[4] = 0;",
              "8 * sizeof(u64), hipHostMallocMapped | hipHostMallocCoherent));\n        for (int k = 0; k < 8; ++k) F.h_plan[k] = 0;")
for k in range(6):
    s = s.replace(f"F.h_plan[{k}]", f"plan_val(F, {k})")
s = s.replace("__atomic_load_n(&plan_val(F, 4), __ATOMIC_ACQUIRE) != want", "!plan_ready(F, want)")
assert s.count("!plan_ready(F, want)") == 2
helpers = '''static bool plan_ready(const TriScratch::FreeSet& F, u32 seq) {
    for (int k = 0; k < 6; ++k)
        if ((u32)(__atomic_load_n(&F.h_plan[k], __ATOMIC_ACQUIRE) >> 32) != seq) return false;
    return true;
}
static u32 plan_val(const TriScratch::FreeSet& F, int k) { return (u32)__atomic_load_n(&F.h_plan[k], __ATOMIC_ACQUIRE); }

'''
s = s.replace("static bool free_enqueue(", helpers + "static bool free_enqueue(", 1)
open(p, "w").write(s)
print("patched", d)
