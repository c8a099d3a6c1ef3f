"""Debug: finds the first op of a primitive-mix scene where the recorded
(command list) and/or immediate GPU results diverge from the oracle."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import scenes

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 32
kw = dict(W=333, H=157, alpha=False, seed=seed, flushes=seed == 33)
rec, imm, ora = scenes.GpuRecordingFactory(), scenes.GpuFactory(), scenes.OracleFactory()

def diff(fac, n):
    a = scenes.scene_primitive_mix(fac, n=n, **kw)["f64"]
    b = scenes.scene_primitive_mix(ora, n=n, **kw)["f64"]
    return not scenes.bits_equal(a, b)

for name, fac in (("immediate", imm), ("recorded", rec)):
    lo, hi = 0, 600
    if not diff(fac, hi):
        print(name, "no mismatch at n=600"); continue
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if diff(fac, mid): hi = mid
        else: lo = mid
    a = scenes.scene_primitive_mix(fac, n=hi, **kw)["f64"]
    b = scenes.scene_primitive_mix(ora, n=hi, **kw)["f64"]
    print(name, "first divergent op count", hi, scenes.first_mismatch(a, b))
    # replay the rng to name the op
    r = np.random.Generator(np.random.PCG64(seed))
    # mirror of scene_primitive_mix's draws: the op index hi-1
    print("  (see scene_primitive_mix op sequence, op index", hi - 1, ")")
