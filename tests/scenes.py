"""Scene library shared by the oracle tests, the GPU parity tests, smoke()
and the golden-fixture generator.

A scene is a function ``scene(fac) -> dict[str, np.ndarray]`` that draws through
the reference's method surface (RenderContext / Texture of
libNativeCPURendererPybind) obtained from a factory.  Two factories exist:
``OracleFactory`` (the CPU restatement in oracle/, test infrastructure) and
``GpuFactory`` (the HIP library through its Pybind mirror).  Running the same
scene on both and comparing the returned arrays bit for bit is the parity
check.
"""
from __future__ import annotations

import ctypes
import math
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# NR_ORACLE_SO: another build of the same restatement (the ASan/UBSan one,
# tests/test_oracle_sanitized.py)
ORACLE_SO = os.environ.get("NR_ORACLE_SO") or os.path.join(ROOT, "oracle", "build", "liboracle.so")


def build_oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return ORACLE_SO


# ---------------------------------------------------------------------------
# oracle-side mirror of the RenderContext/Texture surface
# ---------------------------------------------------------------------------
class _OracleLib:
    _lib = None

    @classmethod
    def get(cls):
        if cls._lib is None:
            import sys
            sys.path.insert(0, ROOT)
            from libnativecpurenderer_amd import _abi
            cls._lib = _abi.bind(ctypes.CDLL(build_oracle()), _abi.ORACLE_ABI)
        return cls._lib


def _vp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleTexture:
    def __init__(self, lib, ptr):
        self.lib, self._ptr = lib, ptr
        self.width = lib.GetTextureWidth(ptr)
        self.height = lib.GetTextureHeight(ptr)
        self.enableAlpha = lib.GetTextureEnableAlpha(ptr)

    def resample(self, w, h):
        return OracleTexture(self.lib, self.lib.ResampleTexture(self._ptr, w, h))


class OracleContext:
    def __init__(self, w, h, alpha):
        self.lib = _OracleLib.get()
        self.width, self.height, self.enable_alpha = w, h, alpha
        self._ptr = self.lib.CreateRenderContext(w, h, alpha)

    def __del__(self):
        if getattr(self, "_ptr", None):
            self.lib.DestroyRenderContext(self._ptr)
            self._ptr = None

    def __getattr__(self, name):
        table = {
            "fill_color": "FillColor", "apply_transform": "ApplyTransform", "scale": "Scale",
            "rotate": "Rotate", "translate": "Translate", "save_state": "SaveContextState",
            "restore_state": "RestoreContextState", "draw_line": "DrawLine", "draw_rect": "DrawRect",
            "draw_circle": "DrawCircle", "set_transform": "SetTransform",
            "set_color_transform": "SetColorTransform", "apply_color_transform": "ApplyColorTransform",
            "set_pixel": "SetPixel", "set_color": "SetColor", "draw_vertical_grd": "DrawVerticalGrd",
            "apply_pixel": "ApplyPixel",
        }
        if name in table:
            fn = getattr(self.lib, table[name])
            return lambda *a: fn(self._ptr, *a)
        raise AttributeError(name)

    def rotate_degree(self, deg):
        self.rotate(deg * math.pi / 180)

    def draw_texture(self, tex, x, y, w, h):
        self.lib.DrawTexture(self._ptr, tex._ptr, x, y, w, h)

    def draw_splitted_texture(self, tex, x, y, w, h, us, ue, vs, ve):
        self.lib.DrawSplittedTexture(self._ptr, tex._ptr, x, y, w, h, us, ue, vs, ve)

    def draw_vertical_mut_grd(self, x, y, width, height, steps):
        for i, (p, s) in enumerate(steps):
            if i == len(steps) - 1:
                break
            np_, ns = steps[i + 1]
            self.draw_vertical_grd(x, y + height * p, width, height * (np_ - p), *s, *ns)

    def get_transform(self):
        out = (ctypes.c_double * 6)()
        self.lib.GetTransform(self._ptr, ctypes.byref(out))
        return tuple(out)

    def get_inverse_transform(self):
        out = (ctypes.c_double * 6)()
        self.lib.GetInverseTransform(self._ptr, ctypes.byref(out))
        return tuple(out)

    def get_color(self, x, y):
        out = [ctypes.c_double() for _ in range(4)]
        self.lib.GetColor(self._ptr, x, y, *(ctypes.byref(o) for o in out))
        return tuple(o.value for o in out)

    def resize(self, w, h):
        self.lib.ResizeRenderContext(self._ptr, w, h)
        self.width, self.height = w, h

    def as_texure(self):
        return OracleTexture(self.lib, self.lib.CreateTextureFromRenderContext(self._ptr))

    def as_texture_shared(self):
        return OracleTexture(self.lib, self.lib.CreateTextureFromRenderContextShared(self._ptr))

    def get_buffer_numpy(self):
        ipp = 4 if self.enable_alpha else 3
        out = np.empty((self.height, self.width, ipp), dtype=np.float64)
        self.lib.GetBuffer(self._ptr, _vp(out))
        return out

    def get_buffer_as_uint8_numpy(self):
        ipp = 4 if self.enable_alpha else 3
        out = np.empty((self.height, self.width, ipp), dtype=np.uint8)
        self.lib.GetBufferAsUInt8(self._ptr, _vp(out))
        return out

    def set_depth_state(self, test, write=True):
        self.lib.SetDepthState(self._ptr, bool(test), bool(write))

    def clear_depth(self, value=0xFFFFFFFF):
        self.lib.ClearDepth(self._ptr, value)

    def get_depth_buffer(self):
        out = np.empty((self.height, self.width), dtype=np.uint32)
        self.lib.GetDepthBuffer(self._ptr, _vp(out))
        return out

    def draw_triangles(self, xy, rgba, z=None, gouraud=None):
        xy = np.ascontiguousarray(xy, dtype=np.float64).reshape(-1, 6)
        n = xy.shape[0]
        rgba = np.ascontiguousarray(rgba, dtype=np.float64)
        if gouraud is None:
            gouraud = rgba.size == 12 * n and n > 0
        rgba = rgba.reshape(n, 12 if gouraud else 4)
        zp = None
        if z is not None:
            z = np.ascontiguousarray(z, dtype=np.float64).reshape(n, 3)
            zp = _vp(z)
        self.lib.DrawTriangles(self._ptr, _vp(xy), zp, _vp(rgba), n, bool(gouraud))
        self._keep = (xy, rgba, z)

    def last_fragment_count(self):
        return self.lib.OracleLastFragmentCount()


class OracleFactory:
    name = "oracle"

    def context(self, w, h, alpha):
        return OracleContext(w, h, alpha)

    def texture(self, arr):
        lib = _OracleLib.get()
        arr = np.ascontiguousarray(arr)
        h, w, c = arr.shape
        if arr.dtype == np.uint8:
            ptr = lib.CreateTextureUInt8(w, h, c == 4, _vp(arr))
        else:
            arr = arr.astype(np.float64)
            ptr = lib.CreateTexture(w, h, c == 4, _vp(arr))
        return OracleTexture(lib, ptr)


class GpuFactory:
    name = "gpu"

    def __init__(self):
        from libnativecpurenderer_amd import libNativeCPURendererPybind as R
        self.R = R

    def context(self, w, h, alpha):
        return self.R.RenderContext(w, h, alpha)

    def texture(self, arr):
        return self.R.Texture.from_numpy(arr)


class GpuRecordingFactory(GpuFactory):
    """The HIP library with every context recording from creation on: all
    primitive draws of a scene go through the deferred command list and run
    when a readback (or another flushing call) comes."""
    name = "gpu-recording"

    def context(self, w, h, alpha):
        ctx = super().context(w, h, alpha)
        ctx.begin_commands()
        return ctx


class GpuPackedFactory(GpuFactory):
    """The HIP library through PackedCommands: a scene's draw and state calls
    are packed on the host and submitted as one ExecuteCommands array before
    anything else (readbacks, triangles, ...) touches the context; with
    `recording`, inside a command list too (one launch per submission)."""
    name = "gpu-packed"

    def __init__(self, recording=False):
        super().__init__()
        self.recording = recording

    def context(self, w, h, alpha):
        ctx = super().context(w, h, alpha)
        if self.recording:
            ctx.begin_commands()
        return ctx.packed()


# ---------------------------------------------------------------------------
# inputs
# ---------------------------------------------------------------------------
def rng(seed=1234):
    return np.random.Generator(np.random.PCG64(seed))


def pattern_u8(h, w, c, seed=7):
    return rng(seed).integers(0, 256, size=(h, w, c), dtype=np.uint8)


def triangle_soup(n, W, H, spread, seed=1234, gouraud=False, alpha=None, zrange=(0.0, 1.0)):
    """C2/C5-style soup: centroid U[0,W)xU[0,H), vertices =
    centroid + U(-spread, spread)^2, z U[zrange), colour U[0,1)^3, a = 1 or
    U[alpha)."""
    g = rng(seed)
    c = np.stack([g.uniform(0, W, n), g.uniform(0, H, n)], axis=1)
    xy = c[:, None, :] + g.uniform(-spread, spread, size=(n, 3, 2))
    z = g.uniform(zrange[0], zrange[1], size=(n, 3))
    k = 3 if gouraud else 1
    col = g.uniform(0, 1, size=(n, k, 4))
    if alpha is None:
        col[..., 3] = 1.0
    else:
        col[..., 3] = g.uniform(alpha[0], alpha[1], size=(n, k))
    return xy.reshape(n, 6), z, col.reshape(n, 4 * k)


def sphere_mesh(W, H, rows, cols, R_frac=0.45):
    """C3's deterministic displaced UV sphere: rows x cols quad
    grid -> 2*rows*cols triangles, r = R(1 + 0.15 sin5θ sin7φ), orthographic,
    centred, both faces drawn, colour = normal*0.5+0.5, Gouraud, z in [0,1]."""
    R = R_frac * H
    th = np.linspace(0, np.pi, rows + 1)
    ph = np.linspace(0, 2 * np.pi, cols + 1)
    T, Pm = np.meshgrid(th, ph, indexing="ij")
    r = R * (1 + 0.15 * np.sin(5 * T) * np.sin(7 * Pm))
    X = r * np.sin(T) * np.cos(Pm)
    Y = r * np.cos(T)
    Z = r * np.sin(T) * np.sin(Pm)
    nx, ny, nz = np.sin(T) * np.cos(Pm), np.cos(T), np.sin(T) * np.sin(Pm)
    sx = W / 2 + X
    sy = H / 2 - Y
    zz = 0.5 + Z / (2.4 * R)            # in (0, 1)
    col = np.stack([nx * 0.5 + 0.5, ny * 0.5 + 0.5, nz * 0.5 + 0.5, np.ones_like(nx)], axis=-1)

    def v(a, i, j):
        return a[i, j]

    i = np.arange(rows)[:, None].repeat(cols, 1).ravel()
    j = np.arange(cols)[None, :].repeat(rows, 0).ravel()
    quads = [(i, j), (i + 1, j), (i + 1, j + 1), (i, j + 1)]
    tris = [(quads[0], quads[1], quads[2]), (quads[0], quads[2], quads[3])]
    xy_l, z_l, c_l = [], [], []
    for tri in tris:
        xy_l.append(np.stack([np.stack([v(sx, *p), v(sy, *p)], -1) for p in tri], 1))
        z_l.append(np.stack([v(zz, *p) for p in tri], 1))
        c_l.append(np.stack([v(col, *p) for p in tri], 1))
    # interleave the two triangles of each quad so submission order is spatial
    xy = np.stack(xy_l, 1).reshape(-1, 6)
    z = np.stack(z_l, 1).reshape(-1, 3)
    c = np.stack(c_l, 1).reshape(-1, 12)
    return np.ascontiguousarray(xy), np.ascontiguousarray(z), np.ascontiguousarray(c)


# ---------------------------------------------------------------------------
# scenes
# ---------------------------------------------------------------------------
def _out(ctx, depth=False):
    d = {"f64": ctx.get_buffer_numpy(), "u8": ctx.get_buffer_as_uint8_numpy()}
    if depth:
        d["depth"] = ctx.get_depth_buffer()
    return d


def scene_clear(fac, W=37, H=23, alpha=False):
    ctx = fac.context(W, H, alpha)
    ctx.set_color(0.25, 0.25, 0.25, 0.25)
    d1 = ctx.get_buffer_numpy()
    ctx.set_color(0.1, 0.2, 0.3, 0.9)          # non-uniform: SetPixel path (A.6 quirk on RGB)
    out = _out(ctx)
    out["uniform"] = d1
    return out


def scene_rects(fac, W=48, H=40, alpha=True):
    ctx = fac.context(W, H, alpha)
    ctx.set_color(0, 0, 0, 0)
    ctx.draw_rect(2.5, 0, 4, 1, 1, 0, 0, 1)                  # x in [2.5, 6.5] -> {3,4,5} (A.7)
    ctx.draw_rect(2, 3, 4, 3, 0, 1, 0, 1)
    ctx.draw_rect(10, 10, 12, 9, 1, 0, 0, 0.5)
    ctx.draw_rect(14, 12, 12, 9, 0, 1, 0, 0.5)               # two alpha-0.5 rects (A.8)
    ctx.save_state()
    ctx.translate(24, 20)
    ctx.rotate(0.3)
    ctx.apply_color_transform(0.5, 1, 0.75, 0.8)
    ctx.draw_rect(-8, -5, 16, 10, 0.2, 0.4, 0.9, 0.7)
    ctx.scale(0.5, 1.5)
    ctx.draw_rect(-3.3, -2.1, 11.7, 7.9, 0.9, 0.1, 0.3, 1)
    ctx.restore_state()
    ctx.set_color_transform(1, 1, 1, 0.5)
    ctx.draw_rect(-5, 30, 100, 100, 0.3, 0.3, 0.6, 1)        # clipped, alpha via colour transform
    ctx.set_transform(1, 0, 0, 1, 0, 0)
    ctx.fill_color(0.1, 0.05, 0.0, 0.25)
    return _out(ctx)


def scene_textures(fac, W=64, H=48, alpha=True):
    tex = fac.texture(pattern_u8(16, 12, 4, seed=3))
    texf = fac.texture(rng(5).uniform(-0.2, 1.3, size=(9, 7, 4)))
    ctx = fac.context(W, H, alpha)
    ctx.set_color(0, 0, 0, 0)
    ctx.draw_texture(tex, 3.7, 2.2, 20.5, 14.3)              # IsNoTransform fast path
    ctx.draw_texture(tex, -5.5, 30.9, 17, 25)                # negative start, clipped
    ctx.draw_texture(texf, 40, 4, 9, 7)
    ctx.save_state()
    ctx.translate(30, 25)
    ctx.rotate(0.7)                                          # inverse path
    ctx.draw_texture(tex, -10, -6, 20, 12)
    ctx.restore_state()
    ctx.save_state()
    ctx.scale(0.5, 0.5)                                      # down-scale: fast path ignores it (A.4)
    ctx.draw_texture(texf, 60, 10, 14, 10)
    ctx.restore_state()
    ctx.save_state()
    ctx.translate(20, 30)
    ctx.scale(1.5, 1.25)
    ctx.apply_color_transform(0.9, 0.8, 0.7, 0.6)
    ctx.draw_splitted_texture(tex, 0, 0, 12, 10, 0.2, 0.7, 0.1, 0.9)
    ctx.draw_splitted_texture(tex, 13, 2, 7.5, 6, 0.0, 1.0, 0.5, 1.0)
    ctx.restore_state()
    small = tex.resample(5, 7) if hasattr(tex, "resample") else None
    if small is not None:
        ctx.draw_texture(small, 50, 30, 10, 14)
    return _out(ctx)


def scene_shapes(fac, W=80, H=60, alpha=False):
    ctx = fac.context(W, H, alpha)
    ctx.set_color(1, 1, 1, 1)
    ctx.draw_vertical_mut_grd(0, H * 0.6, W, H * 0.4, [
        (0.0, (0, 0, 0, 0.0)), (0.25, (0, 0, 0, 0.3)), (0.5, (0, 0, 0, 0.6)),
        (0.75, (0, 0, 0, 0.9)), (1.0, (0, 0, 0, 1.0))])      # milrenderer.py:872-878
    ctx.draw_circle(20.3, 18.7, 11.2, 1, 1, 0, 0.4)
    ctx.draw_line(3, 4, 70, 50, 3.5, 0, 1, 0, 1)
    ctx.draw_line(75, 5, 10, 55, 1.0, 0.2, 0.3, 0.9, 0.8)
    ctx.save_state()
    ctx.translate(40, 30)
    ctx.rotate_degree(33)
    ctx.scale(1.2, 0.8)
    ctx.draw_circle(5, -3, 9, 0.5, 0.1, 0.9, 1)
    ctx.draw_line(-20, 0, 20, 5, 4, 0.9, 0.2, 0.1, 0.6)
    ctx.draw_vertical_grd(-10, -10, 20, 15, 1, 0, 0, 1, 0, 0, 1, 0.5)
    ctx.restore_state()
    ctx.set_transform(0, 0, 0, 0, 0, 0)                     # singular: inv_det = 1e9 (A.10)
    ctx.draw_line(-1, -1, 1, 1, 2, 0.3, 0.3, 0.3, 0.5)
    return _out(ctx)


def scene_demo(fac, t=0.37, size=64, alpha=True):
    """The reference demo's per-frame draw sequence (Pybind.py:704-717), at
    reduced size (scale(1/4) as in :687), texture resampled to 16x16."""
    S = 4
    ctx = fac.context(size, size, alpha)
    ctx.scale(1 / S, 1 / S)
    tex = fac.texture(pattern_u8(128, 128, 4, seed=11)).resample(16, 16)
    ctx.set_color(1, 1, 1, 1)
    ctx.save_state()
    ctx.apply_color_transform(t % 1, (t + 1.4) % 1, (t + 2.8) % 1, 1)
    base = size * S * 0.75
    w = base * (1 + math.sin(t * 2 * math.pi) / 4)
    h = base * (1 + math.cos(t * 3 * math.pi) / 4)
    ctx.draw_texture(tex, w * 1.5 / 2, h * 1.3 / 2, w, h)
    ctx.draw_line(w * 0.1, h * 0.1, w, h, (w + h) / 300, 0, 1, 0, 1)
    ctx.draw_circle(w * 0.3, h * 0.3, 100, 1, 1, 0, 0.4)
    ctx.draw_rect(w * 0.6, h * 0.6, w * 0.1, h * 0.1, 0, 1, 0, 0.4)
    ctx.restore_state()
    return _out(ctx)


def scene_primitive_mix(fac, W=96, H=72, alpha=False, n=160, seed=21, flushes=False, apply_px=True):
    """A milrenderer-style frame (milrenderer.py:865-1038 mix): seeded random
    sequence of every primitive under changing transforms, colour transforms
    and saved states, with single-pixel ops.  flushes=True adds calls that
    must run queued draws first (get_color, a framebuffer snapshot drawn
    back) and a mid-sequence set_color.  apply_px=False leaves out
    apply_pixel, which the reference binding cannot call (not exported,
    SURVEY §8b)."""
    r = np.random.Generator(np.random.PCG64(seed))
    ctx = fac.context(W, H, alpha)
    ctx.set_color(0.1, 0.1, 0.1, 0.1)
    tex_a = fac.texture(pattern_u8(24, 20, 4, seed=seed + 1))
    tex_b = fac.texture(pattern_u8(9, 13, 3, seed=seed + 2))
    probes = []

    def col():
        return [float(v) for v in r.uniform(0, 1, 3)] + [float(r.choice([1.0, r.uniform(0.2, 0.9)]))]

    for k in range(n):
        op = int(r.integers(0, 13))
        x, y = float(r.uniform(-10, W + 5)), float(r.uniform(-10, H + 5))
        w, h = float(r.uniform(-3, W / 2)), float(r.uniform(-3, H / 2))
        if op == 0:
            ctx.draw_rect(x, y, w, h, *col())
        elif op == 1:
            ctx.draw_texture(tex_a if r.uniform() < 0.5 else tex_b, x, y, w, h)
        elif op == 2:
            ctx.draw_splitted_texture(tex_a, x, y, w, h, *[float(v) for v in r.uniform(0, 1, 4)])
        elif op == 3:
            ctx.draw_line(x, y, float(r.uniform(0, W)), float(r.uniform(0, H)), float(r.uniform(0.5, 6)), *col())
        elif op == 4:
            ctx.draw_circle(x, y, float(r.uniform(0.5, 15)), *col())
        elif op == 5:
            ctx.draw_vertical_grd(x, y, w, h, *col(), *col())
        elif op == 6 and apply_px:
            ctx.apply_pixel(int(r.integers(-2, W + 2)), int(r.integers(-2, H + 2)), *col())
        elif op == 7:
            px = int(r.integers(0, W)) if r.uniform() < 0.8 else W - 1
            ctx.set_pixel(px, int(r.integers(0, H)), *col())
        elif op == 8:
            ctx.save_state()
            ctx.translate(float(r.uniform(-20, 20)), float(r.uniform(-20, 20)))
            ctx.rotate(float(r.uniform(-0.5, 0.5)))
            ctx.scale(float(r.uniform(0.5, 1.5)), float(r.uniform(0.5, 1.5)))
        elif op == 9:
            ctx.restore_state()
        elif op == 10:
            ctx.apply_color_transform(*[float(v) for v in r.uniform(0.7, 1.1, 4)])
        elif op == 11:
            if r.uniform() < 0.2:
                ctx.fill_color(*col())
            else:
                ctx.set_color_transform(1, 1, 1, 1)
        elif op == 12 and flushes:
            m = int(r.integers(0, 3))
            if m == 0:
                probes.append(ctx.get_color(float(r.uniform(0, W)), float(r.uniform(0, H))))
            elif m == 1:
                snap = ctx.as_texure()
                ctx.draw_texture(snap, x, y, w, h)
            else:
                v = float(r.uniform(0, 1))
                ctx.set_color(v, v, v, v)
    out = _out(ctx)
    if probes:
        out["probes"] = np.array(probes, dtype=np.float64)
    return out


def scene_render_to_texture(fac, W=40, H=30):
    ctx = fac.context(W, H, True)
    ctx.set_color(0, 0, 0, 0)
    ctx.draw_rect(5, 5, 20, 12, 0.8, 0.3, 0.1, 1)
    snap = ctx.as_texure()
    shared = ctx.as_texture_shared()
    ctx2 = fac.context(W, H, True)
    ctx2.set_color(0.5, 0.5, 0.5, 0.5)
    ctx2.draw_texture(snap, 3, 4, 30, 20)
    ctx2.draw_texture(shared, 10, 2, 12, 9)
    return _out(ctx2)


def scene_u8(fac):
    ctx = fac.context(8, 2, False)
    vals = [1.8, 1.2, 2.4, -0.5, 0.999, 1.0, 0.5, 1e12, -1e12, 255.0, 3.0, -0.003]
    ctx.set_color(0, 0, 0, 0)
    for k in range(len(vals) // 4):
        ctx.set_pixel(2 * k + 1, 1, vals[4 * k], vals[4 * k + 1], vals[4 * k + 2], vals[4 * k + 3])
    return _out(ctx)


def scene_triangles(fac, W=70, H=50, alpha=False, n=300, spread=9.0, seed=1, gouraud=False,
                    depth=True, depth_write=True, alpha_range=None, transform=False):
    xy, z, rgba = triangle_soup(n, W, H, spread, seed=seed, gouraud=gouraud, alpha=alpha_range)
    ctx = fac.context(W, H, alpha)
    ctx.set_color(0, 0, 0, 0)
    if depth:
        ctx.set_depth_state(True, depth_write)
        ctx.clear_depth()
    if transform:
        ctx.translate(W / 2, H / 2)
        ctx.rotate(0.4)
        ctx.scale(0.9, 1.1)
        ctx.translate(-W / 2, -H / 2)
        ctx.apply_color_transform(0.9, 1.0, 0.8, 1.0)
    ctx.draw_triangles(xy, rgba, z=z, gouraud=gouraud)
    return _out(ctx, depth=depth)


def scene_triangle_edges(fac, W=70, H=66, alpha=True):
    """Hand-built edge cases: integer vertices on pixel centres, shared
    edges, horizontal edges, slivers, zero area, non-finite, huge coords,
    tile-boundary crossings (64x32 tiles), a fan."""
    T = []
    T.append([2, 2, 10, 2, 2, 10])            # right angle, integer vertices
    T.append([10, 2, 10, 10, 2, 10])          # shares the hypotenuse
    T.append([20, 5, 30, 5, 25, 5])           # zero area
    T.append([60, 30, 68, 30, 64, 40])        # crosses the x=64 and y=32 tile edges
    T.append([0.5, 40.5, 40.25, 41.75, 3.1, 65.9])
    T.append([-1e9, 20, 1e9, 21, 35, 60])     # huge coordinates
    T.append([float("nan"), 1, 2, 3, 4, 5])   # non-finite: skipped
    T.append([45, 45, 45.2, 60, 45.1, 45])    # sliver
    T.append([33, 33, 33, 33, 40, 40])        # degenerate (repeated vertex)
    T.append([50, 10, 69, 0, 69, 20])
    T.append([64, 32, 63, 31, 65, 31])        # tiny, on the tile corner
    for k in range(8):                         # fan around (20, 50)
        a0, a1 = k * math.pi / 4, (k + 1) * math.pi / 4
        T.append([20, 50, 20 + 12 * math.cos(a0), 50 + 12 * math.sin(a0),
                  20 + 12 * math.cos(a1), 50 + 12 * math.sin(a1)])
    xy = np.array(T, dtype=np.float64)
    n = len(T)
    g = rng(9)
    rgba = g.uniform(0, 1, size=(n, 12))
    rgba[:, 3::4] = g.uniform(0.3, 1.0, size=(n, 3))
    rgba[0, 3::4] = 1.0
    z = g.uniform(0, 1, size=(n, 3))
    z[1] = [-0.5, 1.5, 0.5]                    # out-of-range depths clamp
    ctx = fac.context(W, H, alpha)
    ctx.set_color(0.1, 0.1, 0.1, 0.1)
    ctx.set_depth_state(True, True)
    ctx.clear_depth(0xFFFFFFF0)
    ctx.draw_triangles(xy, rgba, z=z, gouraud=True)
    ctx.set_depth_state(False, False)
    ctx.draw_triangles(xy[:4] + 3.0, rgba[:4, :4], z=None, gouraud=False)
    return _out(ctx, depth=True)


def scene_triangles_multi(fac, W=130, H=97):
    """Several draw calls with state changes in between: the deferred clears,
    depth write off, colour transforms and a texture draw interleaved."""
    ctx = fac.context(W, H, False)
    ctx.set_color(0.2, 0.2, 0.2, 0.2)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    xy, z, c = triangle_soup(400, W, H, 12, seed=21, gouraud=True)
    ctx.draw_triangles(xy, c, z=z)
    ctx.draw_rect(10, 10, 40, 30, 0.9, 0.1, 0.1, 0.5)
    ctx.set_depth_state(True, False)
    xy2, z2, c2 = triangle_soup(200, W, H, 30, seed=22, alpha=(0.2, 0.8))
    ctx.save_state()
    ctx.apply_color_transform(0.7, 0.9, 1.0, 0.9)
    ctx.draw_triangles(xy2, c2, z=z2)
    ctx.restore_state()
    ctx.set_depth_state(False, False)
    ctx.clear_depth(12345)
    xy3, z3, c3 = triangle_soup(50, W, H, 20, seed=23, alpha=(0.5, 1.0))
    ctx.draw_triangles(xy3, c3)
    ctx.set_color(0, 0, 0, 0)
    ctx.draw_triangles(xy3[:10], c3[:10])
    return _out(ctx, depth=True)


TRIANGLE_SCENES = {
    "tri_flat_depth": dict(),
    "tri_flat_painter": dict(depth=False, seed=2),
    "tri_gouraud_depth_rgba": dict(alpha=True, gouraud=True, seed=3),
    "tri_blend_ztest_nowrite": dict(depth_write=False, alpha_range=(0.2, 0.8), seed=4, spread=20.0),
    "tri_transform": dict(transform=True, gouraud=True, seed=5, alpha_range=(0.5, 1.0)),
    "tri_ragged_big": dict(W=131, H=77, n=2000, spread=6.0, seed=6, gouraud=True),
    "tri_large_overdraw": dict(W=100, H=70, n=150, spread=60.0, seed=7, alpha_range=(0.2, 0.8),
                               depth_write=False),
}

BASIC_SCENES = {
    "clear_rgb": (scene_clear, dict(alpha=False)),
    "clear_rgba": (scene_clear, dict(alpha=True)),
    "rects_rgba": (scene_rects, dict(alpha=True)),
    "rects_rgb": (scene_rects, dict(alpha=False)),
    "textures_rgba": (scene_textures, dict(alpha=True)),
    "textures_rgb": (scene_textures, dict(alpha=False)),
    "shapes_rgb": (scene_shapes, dict(alpha=False)),
    "shapes_rgba": (scene_shapes, dict(alpha=True)),
    "demo_t037": (scene_demo, dict(t=0.37)),
    "demo_t081": (scene_demo, dict(t=0.81)),
    "render_to_texture": (scene_render_to_texture, dict()),
    "mix_rgb": (scene_primitive_mix, dict(alpha=False, apply_px=False)),
    "mix_rgba": (scene_primitive_mix, dict(alpha=True, seed=22, apply_px=False)),
    "mix_px_flush_rgb": (scene_primitive_mix, dict(alpha=False, seed=23, flushes=True)),
    "mix_px_flush_rgba": (scene_primitive_mix, dict(alpha=True, seed=24, flushes=True, n=220)),
    "u8": (scene_u8, dict()),
    "tri_edges": (scene_triangle_edges, dict()),
    "tri_multi": (scene_triangles_multi, dict()),
}


def all_scenes():
    d = dict(BASIC_SCENES)
    for k, kw in TRIANGLE_SCENES.items():
        d[k] = (scene_triangles, kw)
    return d


def run_scene(name, fac):
    fn, kw = all_scenes()[name]
    return fn(fac, **kw)


def bits_equal(a: np.ndarray, b: np.ndarray) -> bool:
    """Bit-for-bit equality (distinguishes -0.0/+0.0 and NaN payloads)."""
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    if a.dtype == np.float64:
        return np.array_equal(a.view(np.uint64), b.view(np.uint64))
    return np.array_equal(a, b)


def first_mismatch(a, b):
    if a.shape != b.shape:
        return f"shape {a.shape} != {b.shape}"
    va = a.view(np.uint64) if a.dtype == np.float64 else a
    vb = b.view(np.uint64) if b.dtype == np.float64 else b
    idx = np.argwhere(va != vb)
    if len(idx) == 0:
        return None
    i = tuple(idx[0])
    return f"{len(idx)} mismatches, first at {i}: {a[i]!r} vs {b[i]!r}"


# ---------------------------------------------------------------------------
# hit-effect texture (cpp:1318-1440) on both sides
# ---------------------------------------------------------------------------
def hit_mask(w, h, seed=7):
    """Seeded RGBA u8 mask (non-square shapes exercise the column-major
    indexing of cpp:1413-1432)."""
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8)


def oracle_hit_effect(mask_u8, seed, t, rgb=(0x96 / 0xff, 0x90 / 0xff, 0xfd / 0xff)):
    lib = _OracleLib.get()
    h, w, _ = mask_u8.shape
    m = lib.CreateTextureUInt8(w, h, True, _vp(np.ascontiguousarray(mask_u8)))
    tex = lib.CreateMilthmHitEffectTexture(m, seed, t, *rgb)
    out = np.empty((h, w, 4), dtype=np.float64)
    lib.OracleGetTextureBuffer(tex, _vp(out))
    lib.DestroyTexture(tex)
    lib.DestroyTexture(m)
    return out


# ---------------------------------------------------------------------------
# YUV420P restatement (GetFrameYUV420P; swscale's unscaled rgb24toyv12 path)
# ---------------------------------------------------------------------------
YUV_COEF = ((8414, 16519, 3208), (-4864, -9527, 14392), (14392, -12060, -2331))


def yuv420p(rgb_u8):
    """(H, W, 3|4) u8 frame -> flat Y | U | V planes: BT.601 limited range,
    15-bit coefficients, (c . rgb >> 15) + 16/128/128 (arithmetic shift),
    chroma taken at the top-left pixel of each 2x2 block."""
    h, w = rgb_u8.shape[:2]
    p = rgb_u8[..., :3].astype(np.int64)
    r, g, b = p[..., 0], p[..., 1], p[..., 2]
    (ry, gy, by), (ru, gu, bu), (rv, gv, bv) = YUV_COEF
    y = ((ry * r + gy * g + by * b) >> 15) + 16
    rs, gs, bs = r[0::2, 0::2], g[0::2, 0::2], b[0::2, 0::2]
    u = ((ru * rs + gu * gs + bu * bs) >> 15) + 128
    v = ((rv * rs + gv * gs + bv * bs) >> 15) + 128
    return np.concatenate([y.ravel(), u.ravel(), v.ravel()]).astype(np.uint8)
