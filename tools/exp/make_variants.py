"""Builds ablation variants of the order-free raster into tools/exp/<name>.so
(A/B timing only; never shipped).  Each variant removes one stage of k_vis so
the per-stage cost is the difference of two bench lines:
  e0 full   e1 no shading (depth only)   e2 + no pixel loop   e3 + no row loop
Other variants: name=DEF=VAL+DEF2=VAL (compile-time knobs, e.g. NR_VWG).
Usage: python tools/exp/make_variants.py [names...]; run with tools/exp/run.sh."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(ROOT, "libnativecpurenderer_amd", "csrc")
VARIANTS = {
    "e0": [],
    "e1": ["EXP_NOSHADE"],
    "e2": ["EXP_NOSHADE", "EXP_NOPIX"],
    "e3": ["EXP_NOSHADE", "EXP_NOITEMS"],
}
PATCHES = [
    ("            for (int it = lane; it < R; it += 64) {",
     "            for (int it = lane; it < (EXP_NOITEMS ? 0 : R); it += 64) {"),
    ("                if (COUNT) myFrags += (unsigned long long)(xe - xs);",
     "                if (COUNT) myFrags += (unsigned long long)(xe - xs);\n"
     "                if (EXP_NOPIX) { if (xe > 100) key[0] = xe; continue; }"),
    ("                if (lx < wlim && ly < hlim) resolve_pixel<ZMODE, GOURAUD>(fp, x0 + lx, y0 + ly, key[p]);",
     "                if (EXP_NOSHADE) { if (lx < wlim && ly < hlim) fp.depth[(y0+ly)*fp.W+x0+lx] = (u32)key[p]; continue; }\n"
     "                if (lx < wlim && ly < hlim) resolve_pixel<ZMODE, GOURAUD>(fp, x0 + lx, y0 + ly, key[p]);"),
]


def main(names):
    src = open(os.path.join(SRC, "nr_tri_free.hip")).read()
    for a, b in PATCHES:
        assert src.count(a) == 1, a
        src = src.replace(a, b)
    src = "#ifndef EXP_NOITEMS\n#define EXP_NOITEMS 0\n#endif\n#ifndef EXP_NOPIX\n#define EXP_NOPIX 0\n#endif\n" \
          "#ifndef EXP_NOSHADE\n#define EXP_NOSHADE 0\n#endif\n" + src
    tmp = os.path.join(SRC, "_exp_tri_free.hip")
    open(tmp, "w").write(src)
    objs = [os.path.join(ROOT, "build", "obj", f) for f in sorted(os.listdir(os.path.join(ROOT, "build", "obj")))
            if f.endswith(".o") and f != "nr_tri_free.o"]
    procs = []
    try:
        for n in names:
            if "=" in n:
                n, spec = n.split("=", 1)
                defs = [f"-D{d}" for d in spec.split("+")]
            else:
                defs = [f"-D{d}=1" for d in VARIANTS[n]]
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
