"""Phase clocks of the ordered raster (k_tile_raster): builds tools/exp/oph.so
with s_memrealtime stamps (100 MHz) at the chunk phase boundaries of every
workgroup -- setup (records -> LDS), spans, blend -- summed into g_acc, then
(with `run`) renders C5 frames with it and prints the per-phase workgroup time.
Usage: python tools/exp/ordered_phases.py build | run"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "libnativecpurenderer_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools", "exp"))

PATCHES = [
    ("    for (u32 base = ls; base < le; base += CH) {\n",
     "    u64 ph_a = 0, ph_b = 0, ph_c = 0, ph_n = 0, ph_t = 0;\n    const u64 ph_k0 = __builtin_amdgcn_s_memrealtime();\n"
     "    for (u32 base = ls; base < le; base += CH) {\n        ph_t = __builtin_amdgcn_s_memrealtime(); ++ph_n;\n"),
    ("        const bool allBlend = __syncthreads_and(blendOnly ? 1 : 0) != 0;\n",
     "        const bool allBlend = __syncthreads_and(blendOnly ? 1 : 0) != 0;\n"
     "        { const u64 x = __builtin_amdgcn_s_memrealtime(); ph_a += x - ph_t; ph_t = x; }\n"),
    ("        __syncthreads();\n        // this wave's triangles of the chunk",
     "        __syncthreads();\n        { const u64 x = __builtin_amdgcn_s_memrealtime(); ph_b += x - ph_t; ph_t = x; }\n"
     "        // this wave's triangles of the chunk"),
    ("            __syncthreads();\n            continue;\n",
     "            __syncthreads();\n            { const u64 x = __builtin_amdgcn_s_memrealtime(); ph_c += x - ph_t; ph_t = x; }\n"
     "            continue;\n"),
    ("        __syncthreads();\n    }\n\n    // ---- write the tile back once\n",
     "        __syncthreads();\n        { const u64 x = __builtin_amdgcn_s_memrealtime(); ph_c += x - ph_t; ph_t = x; }\n    }\n"
     "    const u64 ph_k1 = __builtin_amdgcn_s_memrealtime();\n\n    // ---- write the tile back once\n"),
    ("    if (COUNT) {\n        atomicAdd(&fragSum, myFrags);",
     "    if (tid == 0) { atomicAdd(&g_acc[0], ph_a); atomicAdd(&g_acc[1], ph_b); atomicAdd(&g_acc[2], ph_c);\n"
     "        atomicAdd(&g_acc[3], ph_n); atomicAdd(&g_acc[4], ph_k1 - ph_k0);\n"
     "        atomicAdd(&g_acc[5], __builtin_amdgcn_s_memrealtime() - ph_k1); atomicAdd(&g_acc[6], 1ull); }\n"
     "    if (COUNT) {\n        atomicAdd(&fragSum, myFrags);"),
]


def build():
    import make_variants as mv
    src = open(os.path.join(SRC, "nr_tri_ordered.hip")).read()
    for a, b in PATCHES:
        assert src.count(a) == 1, a
        src = src.replace(a, b)
    tmp = os.path.join(SRC, "_exp_ordered.hip")
    open(tmp, "w").write(mv.PRELUDE + src + mv.HOST)
    objs = [os.path.join(ROOT, "build", "obj", f) for f in sorted(os.listdir(os.path.join(ROOT, "build", "obj")))
            if f.endswith(".o") and f != "nr_tri_ordered.o"]
    try:
        subprocess.check_call(
            f"/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-gpu-rdc "
            f"-Wno-pass-failed -I{SRC} -c {tmp} -o /tmp/_oph.o && /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared "
            f"-fPIC -o {ROOT}/tools/exp/oph.so {' '.join(objs)} /tmp/_oph.o -ldl", shell=True)
    finally:
        os.remove(tmp)


def run():
    import numpy as np
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    from libnativecpurenderer_amd import _lib
    _lib.LIB_PATH = os.path.join(ROOT, "tools", "exp", "oph.so")   # (the phase-clock build)
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    cfg = bench.CONFIGS[sys.argv[2] if len(sys.argv) > 2 else "c5"]
    xy, z, c = bench.make_scene(cfg)
    ctx = R.RenderContext(cfg["W"], cfg["H"], False)
    buf = R.TriangleBuffer(xy, c, z=z)
    lib = _lib.load()
    acc = np.zeros(8, np.uint64)
    for it in range(3):
        lib.ExpResetAcc()
        ctx.set_color(0, 0, 0, 0)
        ctx.set_depth_state(True, cfg.get("write", True))
        ctx.clear_depth()
        ctx.draw_triangle_buffer(buf)
        ctx.flush()
    lib.ExpGetAcc(acc.ctypes.data_as(ctypes.c_void_p))
    a = acc.astype(np.float64) / 100.0   # us of workgroup time
    nwg = max(1, acc[6])
    print(f"workgroups {acc[6]}  chunks {acc[3]}  per WG: chunk loop {a[4]/nwg:.1f} us (setup {a[0]/nwg:.1f}, spans "
          f"{a[1]/nwg:.1f}, blend {a[2]/nwg:.1f}), write-back {a[5]/nwg:.2f} us; per chunk: setup {a[0]/acc[3]:.3f} "
          f"spans {a[1]/acc[3]:.3f} blend {a[2]/acc[3]:.3f} us")


if __name__ == "__main__":
    build() if sys.argv[1] == "build" else run()
