"""Builds ablation / instrumentation variants of the order-free raster into
tools/exp/<name>.so (A/B timing only; never shipped).  Named variants:
  e1 no shading of single-slice tiles   e2 + no pixel loop   e3 + no row loop   e4 + no raster
  times  per-work-item start/end clocks (ExpGetItemTimes, tools/exp/item_times.py)
Other variants: name=DEF=VAL+DEF2=VAL (compile-time knobs, e.g. NR_VWG, NR_SLICE).
Usage: python tools/exp/make_variants.py [names...]; load one with bench.py --lib tools/exp/<name>.so."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "libnativecpurenderer_amd", "csrc")
VARIANTS = {
    "e1": ["EXP_NOSHADE"],
    "e2": ["EXP_NOSHADE", "EXP_NOPIX"],
    "e3": ["EXP_NOSHADE", "EXP_NOROWS"],
    "e4": ["EXP_NOSHADE", "EXP_NORASTER"],
    "na": ["EXP_NOATOMIC"],
    "nf64": ["EXP_NOF64ST"],
    "nu8": ["EXP_NOU8ST"],
    "nst": ["EXP_NOF64ST", "EXP_NOU8ST"],
    "plant": ["EXP_PLANT"],
    "times": ["EXP_TIMES"],
    "planr": ["EXP_PLANR"],
    "binph": ["EXP_BINPH"],
    "warmph": ["EXP_WARMPH"],
    "norsv": ["EXP_NORSV"],
    "sht": ["EXP_SHT"],
    "nosum": ["EXP_NOSUM"],
}
# define -> [(anchor, replacement)]; only the patches of the defines in use are applied
PATCHES = {
    "EXP_NOSUM": [   # no pair-sum atomic in k_bin_warm (and no sum check in k_vis): its cost
        ("    if (tid == 0 && wgPairs) atomicAdd(&wstat[WS_SUM], wgPairs);\n", "\n"),
        ("        fb = !plan[3] || wt == wc.tag || ws != wc.expect;\n", "        fb = !plan[3] || wt == wc.tag;\n"),
    ],
    "EXP_BINPH": [   # per-WG phase durations of k_free_count / k_free_emit -> g_acc[0..3] (count), g_acc[4..6] (emit), spans g_exp
        ("    f64 pxy[TPT][6];\n#pragma unroll\n    for (int k = 0; k < TPT; ++k) {\n        const i64 t = base + k * 256 + tid;\n        if (t < bp.src.n) load_tri_xy(bp.src.xy, t, pxy[k]);\n    }\n",
         "    const u64 c_t0 = __builtin_amdgcn_s_memrealtime();\n    f64 pxy[TPT][6];\n#pragma unroll\n    for (int k = 0; k < TPT; ++k) {\n        const i64 t = base + k * 256 + tid;\n        if (t < bp.src.n) load_tri_xy(bp.src.xy, t, pxy[k]);\n    }\n"
         "    __builtin_amdgcn_s_waitcnt(0);\n    const u64 c_t1 = __builtin_amdgcn_s_memrealtime();\n"),
        ("    if (LDSH) {\n        for (int b = tid; b < ntiles; b += 256) hist[b] = 0;\n        __syncthreads();\n    }\n#pragma unroll\n",
         "    if (LDSH) {\n        for (int b = tid; b < ntiles; b += 256) hist[b] = 0;\n        __syncthreads();\n    }\n    const u64 c_t2 = __builtin_amdgcn_s_memrealtime();\n#pragma unroll\n"),
        ("    if (LDSH) {\n        __syncthreads();\n        for (int b = tid; b < ntiles; b += 256) {\n            const u32 h = hist[b];\n            if (h) atomicAdd(&tile_cnt[b], h);\n        }\n    }\n}",
         "    if (LDSH) {\n        __syncthreads();\n        const u64 c_t3 = __builtin_amdgcn_s_memrealtime();\n        for (int b = tid; b < ntiles; b += 256) {\n            const u32 h = hist[b];\n            if (h) atomicAdd(&tile_cnt[b], h);\n        }\n"
         "        __builtin_amdgcn_s_waitcnt(0);\n        __syncthreads();\n        if (tid == 0) { const u64 c_t4 = __builtin_amdgcn_s_memrealtime();\n"
         "            atomicAdd(&g_acc[0], c_t1 - c_t0); atomicAdd(&g_acc[1], c_t2 - c_t1); atomicAdd(&g_acc[2], c_t3 - c_t2); atomicAdd(&g_acc[3], c_t4 - c_t3);\n"
         "            atomicAdd(&g_acc[7], 1ull); atomicMin(&g_exp[0], c_t0); atomicMax(&g_exp[1], c_t4); }\n    }\n}"),
    ],
    "EXP_PLANR": [   # s_memrealtime stamps at k_free_plan_r's phase boundaries -> g_exp[8*slot + 0..5]
        ("    const int per = (((ntiles + T - 1) / T) + 3) & ~3;\n",
         "    const u64 pr0 = __builtin_amdgcn_s_memrealtime();\n    const int per = (((ntiles + T - 1) / T) + 3) & ~3;\n"),
        ("    const u32 ia = wave_scan(a, lane), ih = wave_scan(hv, lane);\n",
         "    __builtin_amdgcn_s_waitcnt(0);\n    const u64 pr1 = __builtin_amdgcn_s_memrealtime();\n    const u32 ia = wave_scan(a, lane), ih = wave_scan(hv, lane);\n"),
        ("    const u32 ib = wave_scan(b, lane), im = wave_scan(m, lane);\n",
         "    const u64 pr2 = __builtin_amdgcn_s_memrealtime();\n    const u32 ib = wave_scan(b, lane), im = wave_scan(m, lane);\n"),
        ("    {   // c[j] becomes tile j's list offset\n",
         "    const u64 pr3 = __builtin_amdgcn_s_memrealtime();\n    {   // c[j] becomes tile j's list offset\n"),
        ("    if (tid == 0) {\n        off[ntiles] = ta;   // (the same",
         "    __builtin_amdgcn_s_waitcnt(0);\n    __syncthreads();\n    const u64 pr4 = __builtin_amdgcn_s_memrealtime();\n    if (tid == 0) {\n        off[ntiles] = ta;   // (the same"),
        ("        __hip_atomic_store(&host_totals[4], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);\n    }\n}\n\n// NR_PLAN_REG",
         "        __hip_atomic_store(&host_totals[4], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);\n"
         "        __builtin_amdgcn_s_waitcnt(0);\n        const u64 pr5 = __builtin_amdgcn_s_memrealtime();\n        const u64 slot = atomicAdd(&g_acc[7], 1ull) % 4096;\n        g_exp[8 * slot] = pr0; g_exp[8 * slot + 1] = pr1; g_exp[8 * slot + 2] = pr2; g_exp[8 * slot + 3] = pr3; g_exp[8 * slot + 4] = pr4; g_exp[8 * slot + 5] = pr5; g_exp[8 * slot + 6] = T;\n    }\n}\n\n// NR_PLAN_REG"),
    ],
    "EXP_TIMES": [
        ("    for (u32 item = blockIdx.x; item < nitems; item += gridDim.x) {\n",
         "    u64 exp_t0 = 0, exp_mid = 0; u32 exp_prev = ~0u; u64 exp_info = 0;\n"
         "    for (u32 item = blockIdx.x; item < nitems; item += gridDim.x) {\n"
         "        if (tid == 0) { const u64 now = __builtin_amdgcn_s_memrealtime();\n"
         "            if (exp_prev != ~0u) exp_record(exp_prev, exp_t0, now, exp_info, exp_mid);\n"
         "            exp_prev = item; exp_t0 = now; exp_mid = 0; const uint4 dd = items[item];\n"
         "            exp_info = (u64)(dd.z - dd.y) | ((u64)dd.w << 32) | ((u64)blockIdx.x << 48); }\n"),
        ("    }   // work items\n",
         "    }   // work items\n"
         "    if (tid == 0 && exp_prev != ~0u) exp_record(exp_prev, exp_t0, __builtin_amdgcn_s_memrealtime(), exp_info, exp_mid);\n"),
        ("        __syncthreads();\n        if (!multi) {   // the whole list was in this slice: shade now\n",
         "        __syncthreads();\n        if (tid == 0) exp_mid = __builtin_amdgcn_s_memrealtime() - exp_t0;\n"
         "        if (!multi) {   // the whole list was in this slice: shade now\n"),
        # split slices: clock after the merge + slice counter (high word, relative to the item start)
        ("        if (!sLast) continue;\n",
         "        if (tid == 0) exp_mid |= (__builtin_amdgcn_s_memrealtime() - exp_t0) << 32;\n        if (!sLast) continue;\n"),
    ],
    "EXP_SHT": [   # shading phase durations summed over all shade_tile calls -> g_acc (0 hash, 1 records, 2 pixels, 5 overflow pixels)
        ("    for (int i = tid; i < HS; i += NT) ht[i] = 0;\n",
         "    const u64 sh_t0 = __builtin_amdgcn_s_memrealtime();\n    for (int i = tid; i < HS; i += NT) ht[i] = 0;\n"),
        ("    __syncthreads();   // every key read: the records may overwrite them\n",
         "    __syncthreads();   // every key read: the records may overwrite them\n    const u64 sh_t1 = __builtin_amdgcn_s_memrealtime();\n"),
        ("        for (u32 u = tid; u < U; u += NT) make_record<GOURAUD>(fp, (i64)didx[u] - 1, rec + u * St::REC);\n    }\n    __syncthreads();\n",
         "        for (u32 u = tid; u < U; u += NT) make_record<GOURAUD>(fp, (i64)didx[u] - 1, rec + u * St::REC);\n    }\n    __syncthreads();\n"
         "    const u64 sh_t2 = __builtin_amdgcn_s_memrealtime();\n"),
        ("        store_colour(fp, gp, px, py, cr, cg, cb, ca);\n    }\n    // pass 3b",
         "        store_colour(fp, gp, px, py, cr, cg, cb, ca);\n    }\n    __syncthreads();\n    const u64 sh_t3 = __builtin_amdgcn_s_memrealtime();\n    // pass 3b"),
        ("                store_colour(fp, gp, px, py, cr, cg, cb, ca);\n            }\n        }\n    }\n}\n",
         "                store_colour(fp, gp, px, py, cr, cg, cb, ca);\n            }\n        }\n    }\n    __syncthreads();\n"
         "    if (tid == 0) { const u64 sh_t4 = __builtin_amdgcn_s_memrealtime();\n"
         "        atomicAdd(&g_acc[0], sh_t1 - sh_t0); atomicAdd(&g_acc[1], sh_t2 - sh_t1); atomicAdd(&g_acc[2], sh_t3 - sh_t2);\n"
         "        atomicAdd(&g_acc[5], sh_t4 - sh_t3); atomicAdd(&g_acc[3], 1ull); atomicAdd(&g_acc[4], (u64)nU); }\n}\n"),
    ],
    "EXP_WARMPH": [   # per-WG phase durations of k_bin_warm -> g_acc[0..3] (loads, LDS histogram, range reservation, pairs), [7] WGs; span g_exp[0..1]
        ("    if (tid == 0) wgPairs = 0;\n",
         "    if (tid == 0) wgPairs = 0;\n    const u64 w_t0 = __builtin_amdgcn_s_memrealtime();\n"),
        ("    __syncthreads();   // (hist and wgPairs zeroed)\n",
         "    __builtin_amdgcn_s_waitcnt(0);\n    __syncthreads();   // (hist and wgPairs zeroed)\n    const u64 w_t1 = __builtin_amdgcn_s_memrealtime();\n"),
        ("    if (LDSH) {\n        __syncthreads();\n        for (int b = tid; b < hbins; b += 256) {   // reserve each touched tile's range once\n",
         "    __syncthreads();\n    const u64 w_t2 = __builtin_amdgcn_s_memrealtime();\n    if (LDSH) {\n        for (int b = tid; b < hbins; b += 256) {   // reserve each touched tile's range once\n"),
        ("    __syncthreads();   // (LDS ranges reserved; wgPairs complete)\n",
         "    __syncthreads();   // (LDS ranges reserved; wgPairs complete)\n    const u64 w_t3 = __builtin_amdgcn_s_memrealtime();\n"),
        ("                if (slot < end) list[slot] = (u32)t;\n            }\n        }\n    }\n}\n",
         "                if (slot < end) list[slot] = (u32)t;\n            }\n        }\n    }\n"
         "    __builtin_amdgcn_s_waitcnt(0);\n    __syncthreads();\n"
         "    if (tid == 0) { const u64 w_t4 = __builtin_amdgcn_s_memrealtime();\n"
         "        atomicAdd(&g_acc[0], w_t1 - w_t0); atomicAdd(&g_acc[1], w_t2 - w_t1); atomicAdd(&g_acc[2], w_t3 - w_t2);\n"
         "        atomicAdd(&g_acc[3], w_t4 - w_t3); atomicAdd(&g_acc[7], 1ull); atomicMin(&g_exp[0], w_t0); atomicMax(&g_exp[1], w_t4); }\n}\n"),
    ],
    "EXP_NORSV": [   # timing only (wrong lists): k_bin_warm's range reservation without its global atomics
        ("                const u32 start = beg + atomicAdd(&cur[tile], h) - epoch * (end - beg);\n",
         "                const u32 start = EXP_NORSV ? beg : beg + atomicAdd(&cur[tile], h) - epoch * (end - beg);\n"),
    ],
    "EXP_NOROWS": [
        ("            if (r0 < r1 && !big) {\n",
         "            if (EXP_NOROWS && r0 < r1 && !big) { if (r1 > 1000) key[0] = r0; }\n            else if (r0 < r1 && !big) {\n"),
    ],
    "EXP_NOPIX": [
        ("                    if (xs >= xe) continue;\n                    if (ZMODE == 0) {",
         "                    if (xs >= xe) continue;\n                    if (EXP_NOPIX) { if (xe > 100) key[0] = xe; continue; }\n"
         "                    if (ZMODE == 0) {"),
    ],
    "EXP_NOSHADE": [
        ("        if (!multi) {   // the whole list was in this slice: shade now\n",
         "        if (EXP_NOSHADE && !multi) continue;\n        if (!multi) {   // the whole list was in this slice: shade now\n"),
    ],
    "EXP_NOATOMIC": [
        ("                    if (ZMODE == 1) atomicMin(&key[p], ((u64)zq << 32) | id1);",
         "                    if (ZMODE == 1 && EXP_NOATOMIC) key[p] = ((u64)zq << 32) | id1;\n"
         "                    else if (ZMODE == 1) atomicMin(&key[p], ((u64)zq << 32) | id1);"),
    ],
    "EXP_NOF64ST": [   # shading skips the f64 framebuffer stores (u8 frame and depth still written)
        ("    dst[0] = cr; dst[1] = cg; dst[2] = cb;\n    if (ipp == 4) dst[3] = ca;\n",
         "    if (!EXP_NOF64ST) { dst[0] = cr; dst[1] = cg; dst[2] = cb;\n    if (ipp == 4) dst[3] = ca; }\n"),
    ],
    "EXP_NOU8ST": [   # shading skips the u8 frame stores
        ("    if (fp.frameU8) {\n        const int r8 = nr_to_u8(cr)",
         "    if (fp.frameU8 && !EXP_NOU8ST) {\n        const int r8 = nr_to_u8(cr)"),
    ],
    "EXP_PLANT": [   # s_memrealtime stamps at the plan kernel's phase boundaries -> g_exp[0..5]
        ("    if (tid < PLAN_NB) bcnt[tid] = 0;\n    __syncthreads();\n    // pass 1",
         "    const u64 pt0 = __builtin_amdgcn_s_memrealtime();\n    if (tid < PLAN_NB) bcnt[tid] = 0;\n    __syncthreads();\n    // pass 1"),
        ("    __syncthreads();\n    // pass 2: offsets and items\n",
         "    __syncthreads();\n    const u64 pt1 = __builtin_amdgcn_s_memrealtime();\n    // pass 2: offsets and items\n"),
        ("        off[ntiles] = ta;\n",
         "        off[ntiles] = ta;\n        const u64 pt2 = __builtin_amdgcn_s_memrealtime();\n"),
        ("        __hip_atomic_store(&host_totals[4], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);\n    }\n}",
         "        __hip_atomic_store(&host_totals[4], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);\n"
         "        const u64 pt3 = __builtin_amdgcn_s_memrealtime();\n"
         "        g_exp[0] = pt0; g_exp[1] = pt1; g_exp[2] = pt2; g_exp[3] = pt3; g_exp[4] = ntiles;\n    }\n}"),
    ],
    "EXP_NORASTER": [
        ("        for (u32 c = wave; c < nch; c += NWV) {",
         "        for (u32 c = wave; c < (EXP_NORASTER ? 0u : nch); c += NWV) {"),
    ],
}
PRELUDE = """#include <hip/hip_runtime.h>
__device__ unsigned long long g_exp[4 * 65536];
__device__ unsigned long long g_acc[8];
__device__ inline void exp_record(unsigned item, unsigned long long t0, unsigned long long t1, unsigned long long info,
                                  unsigned long long tm = 0) {
    if (item < 65536) { g_exp[4 * item] = t0; g_exp[4 * item + 1] = t1; g_exp[4 * item + 2] = info; g_exp[4 * item + 3] = tm; }
}
"""
HOST = """
extern "C" int ExpGetAcc(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_acc), 64, 0, hipMemcpyDeviceToHost) == hipSuccess ? 8 : -1;
}
extern "C" int ExpResetAcc() {
    unsigned long long z[8] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_acc), z, 64, 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
extern "C" int ExpSetTimes(const unsigned long long* in, int n) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_exp), in, (size_t)n * 8, 0, hipMemcpyHostToDevice) == hipSuccess ? n : -1;
}
extern "C" int ExpGetItemTimes(unsigned long long* out, int n) {
    if (n > 4 * 65536) n = 4 * 65536;
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_exp), (size_t)n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? n : -1;
}
"""


def parse(n):
    if "=" in n:
        n, spec = n.split("=", 1)
        defs = spec.split("+")
        return n, [f"-D{d}" for d in defs], [d.split("=")[0] for d in defs if d.split("=")[0] in PATCHES]
    return n, [f"-D{d}=1" for d in VARIANTS[n]], VARIANTS[n]


def main(names):
    specs = [parse(n) for n in names]
    used = {d for _, _, ds in specs for d in ds}
    src = open(os.path.join(SRC, "nr_tri_free.hip")).read()
    for d in sorted(used):
        for a, b in PATCHES[d]:
            if src.count(a) != 1:
                sys.exit(f"make_variants: anchor for {d} not found (update PATCHES):\n{a}")
            src = src.replace(a, b)
    defaults = "".join(f"#ifndef {d}\n#define {d} 0\n#endif\n" for d in PATCHES)
    src = defaults + PRELUDE + src + HOST
    tmp = os.path.join(SRC, "_exp_tri_free.hip")
    open(tmp, "w").write(src)
    objs = [os.path.join(ROOT, "build", "obj", f) for f in sorted(os.listdir(os.path.join(ROOT, "build", "obj")))
            if f.endswith(".o") and f != "nr_tri_free.o"]
    procs = []
    try:
        for n, defs, _ in specs:
            o = f"/tmp/_exp_{n}.o"
            cmd = (f"/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-rdc "
                   f"{' '.join(defs)} -I{SRC} -c {tmp} -o {o} && /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared "
                   f"-fPIC -o {ROOT}/tools/exp/{n}.so {' '.join(objs)} {o} -ldl")
            procs.append(subprocess.Popen(cmd, shell=True))
        for p in procs:
            assert p.wait() == 0
    finally:
        os.remove(tmp)


if __name__ == "__main__":
    main(sys.argv[1:] or list(VARIANTS))
