"""Config C1 (BASELINE.json configs[0]): a 128x128 RGBA texture drawn as a quad
on a 256x256 RGBA context, through the Python surface (the reference's
libNativeCPURendererPybind classes, SURVEY §8d: "C1 is additionally timed
through the build's Python surface").  One step = set_color + draw_texture on
the fast path (identity, cpp:720-750) + draw_texture on the inverse path (the
rotated variant, cpp:752-779) + the u8 readback (GetBufferAsUInt8, cpp:52-57).

Timed on one GPU (HIP library) and on the CPU oracle through the same Python
calls, bit-exactness of the two outputs checked first.  Prints one JSON line:
steps/s and Mpixels/s of drawn (covered) pixels.  The texture is
tests/golden/image_png_rgba.npy (the reference's test_files/image.png).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(fac, img, steps):
    ctx = fac.context(256, 256, True)
    tex = fac.texture(img)

    def step():
        ctx.set_color(0, 0, 0, 0)
        ctx.draw_texture(tex, 64, 64, 128, 128)
        ctx.save_state()
        ctx.translate(128, 128)
        ctx.rotate(0.3)
        ctx.translate(-128, -128)
        ctx.draw_texture(tex, 64, 64, 128, 128)
        ctx.restore_state()
        return ctx.get_buffer_as_uint8_numpy()

    out = step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dt = (time.perf_counter() - t0) / steps
    return out.tobytes(), ctx.get_buffer_numpy(), dt


def main():
    import scenes
    img = np.load(os.path.join(ROOT, "tests", "golden", "image_png_rgba.npy"))
    gb, gf, gdt = run(scenes.GpuFactory(), img, 2000)
    ob, of, odt = run(scenes.OracleFactory(), img, 200)
    assert gb == ob and scenes.bits_equal(gf, of), "C1: GPU and oracle differ"
    # drawn pixels per step: the identity quad (128^2) + the rotated quad (area 128^2, counted as such)
    px = 2 * 128 * 128
    print(json.dumps({
        "config": "C1: 128x128 RGBA texture quad on 256x256 RGBA (identity + rotated), u8 readback, Python surface",
        "gpu_ms_per_step": round(gdt * 1e3, 4), "cpu_oracle_ms_per_step": round(odt * 1e3, 4),
        "gpu_mpixels_s": round(px / gdt / 1e6, 1), "cpu_mpixels_s": round(px / odt / 1e6, 1),
        "note": "launch/ctypes-bound at this size: 4 calls + one synchronous readback per step; bit-exact checked",
        "cpu_cores": 1}))


if __name__ == "__main__":
    main()
