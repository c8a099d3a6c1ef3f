"""Debug: one pixel of the primitive-mix scene before/after op n on GPU and oracle."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import scenes
seed, n, x, y = (int(v) for v in sys.argv[1:5])
kw = dict(W=333, H=157, alpha=False, seed=seed)
for name, fac in (("gpu", scenes.GpuFactory()), ("oracle", scenes.OracleFactory())):
    for k in (n - 1, n):
        v = scenes.scene_primitive_mix(fac, n=k, **kw)["f64"][y, x]
        print(name, k, [float.hex(float(c)) for c in v])
