"""Generates the committed golden fixtures in tests/golden/ (run here, in the
build container; /root/reference does not exist on the GPU box).

1. refbinding_*.npz — the reference's own ctypes module
   (/root/reference/src/libNativeCPURendererPybind.py, imported unmodified from
   its location) driving the CPU oracle, which is loaded through that module's
   `ctypes.CDLL("./libNativeCPURenderer.so")` (Pybind.py:9) from a scratch
   directory holding a symlink to oracle/build/liboracle.so.  This pins the
   oracle's ABI (symbol names, argument types and order, handle semantics) to
   the reference binding, and the outputs are compared with the same scenes
   driven through tests/scenes.py's OracleFactory.
2. scenes.npz — oracle outputs of every scene in tests/scenes.py, so later
   oracle edits are caught (and so the GPU tests have a fixed target besides
   the live oracle).
3. image_png_rgba.npy — the reference's test asset test_files/image.png
   (Pybind.py:701) decoded to a 128x128x4 u8 array (data, used by config C1).

Usage: python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import importlib.util
import math
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
import scenes  # noqa: E402

REF_SRC = "/root/reference/src/libNativeCPURendererPybind.py"
REF_IMG = "/root/reference/test_files/image.png"


def load_reference_binding():
    so = scenes.build_oracle()
    tmp = tempfile.mkdtemp(prefix="refbind_")
    os.symlink(so, os.path.join(tmp, "libNativeCPURenderer.so"))
    cwd = os.getcwd()
    os.chdir(tmp)
    try:
        spec = importlib.util.spec_from_file_location("ref_pybind", REF_SRC)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        os.chdir(cwd)
    return mod


class RefBindingFactory:
    """tests/scenes.py factory on top of the reference's own classes."""

    def __init__(self, mod):
        self.m = mod

    def context(self, w, h, alpha):
        ctx = self.m.RenderContext(w, h, alpha)
        ipp = 4 if alpha else 3

        def get_buffer_numpy():
            return np.array(ctx.get_buffer(), dtype=np.float64).reshape(h, w, ipp)

        def get_buffer_as_uint8_numpy():
            return np.frombuffer(bytes(ctx.get_buffer_as_uint8()), dtype=np.uint8).reshape(h, w, ipp)

        ctx.get_buffer_numpy = get_buffer_numpy
        ctx.get_buffer_as_uint8_numpy = get_buffer_as_uint8_numpy
        return ctx

    def texture(self, arr):
        arr = np.ascontiguousarray(arr)
        h, w, c = arr.shape
        assert arr.dtype == np.uint8, "the reference binding's f64 path is broken (Pybind.py:391)"
        return self.m.Texture(w, h, c == 4, arr.tobytes())


def ref_binding_scenes():
    """Scenes expressible through the reference binding (u8 textures only,
    no get_color, no triangles)."""
    return {
        "demo_t037": (scenes.scene_demo, dict(t=0.37)),
        "demo_t081": (scenes.scene_demo, dict(t=0.81)),
        "rects_rgba": (scenes.scene_rects, dict(alpha=True)),
        "rects_rgb": (scenes.scene_rects, dict(alpha=False)),
        "shapes_rgb": (scenes.scene_shapes, dict(alpha=False)),
        "clear_rgb": (scenes.scene_clear, dict(alpha=False)),
        "render_to_texture": (scenes.scene_render_to_texture, dict()),
        "mix_rgb": scenes.all_scenes()["mix_rgb"],
        "mix_rgba": scenes.all_scenes()["mix_rgba"],
    }


def main():
    out = {}
    # 1. reference binding -> oracle
    ref = load_reference_binding()
    assert ref.get_version() == 1
    rf = RefBindingFactory(ref)
    of = scenes.OracleFactory()
    for name, (fn, kw) in ref_binding_scenes().items():
        a = fn(rf, **kw)
        b = fn(of, **kw)
        for k in a:
            assert scenes.bits_equal(a[k], b[k]), (name, k, scenes.first_mismatch(a[k], b[k]))
        np.savez_compressed(os.path.join(HERE, f"refbinding_{name}.npz"), **a)
        print("refbinding", name, "ok")

    # 2. oracle outputs of every scene
    digests = []
    for name in scenes.all_scenes():
        res = scenes.run_scene(name, of)
        for k, v in res.items():
            out[f"{name}/{k}"] = v
            digests.append(f"{name}/{k} {hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest()}")
    np.savez_compressed(os.path.join(HERE, "scenes.npz"), **out)
    with open(os.path.join(HERE, "scenes.sha256"), "w") as f:
        f.write("\n".join(digests) + "\n")
    print("scenes", len(out), "arrays")

    # 3. the reference's test image as data
    if os.path.exists(REF_IMG):
        from PIL import Image
        img = np.array(Image.open(REF_IMG).convert("RGBA"), dtype=np.uint8)
        np.save(os.path.join(HERE, "image_png_rgba.npy"), img)
        print("image", img.shape)


if __name__ == "__main__":
    main()
