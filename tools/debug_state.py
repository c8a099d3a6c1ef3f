"""Debug: transform state of the primitive-mix scene after n ops, GPU vs oracle."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import scenes
seed, n = int(sys.argv[1]), int(sys.argv[2])
for name, fac in (("gpu", scenes.GpuFactory()), ("oracle", scenes.OracleFactory())):
    keep = {}
    orig = fac.context
    def ctxf(w, h, a, orig=orig):
        c = orig(w, h, a); keep["c"] = c; return c
    fac.context = ctxf
    scenes.scene_primitive_mix(fac, n=n, W=333, H=157, alpha=False, seed=seed)
    c = keep["c"]
    print(name, "m", [float.hex(v) for v in c.get_transform()])
    print(name, "inv", [float.hex(v) for v in c.get_inverse_transform()])
