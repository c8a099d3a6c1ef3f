"""CPU tests of the oracle (test infrastructure): pinned against the reference
behaviours recorded in SURVEY.md Appendix A (observed on the reference build
during the survey), against the reference's own ctypes binding
(tests/golden/refbinding_*.npz, made by tests/golden/make_golden.py), and
against the committed scene fixtures.  Also checks, on the CPU, that the
per-row span rule used by the GPU raster is identical to the per-pixel
even-odd test of cpp:822-845."""
import hashlib
import math
import os

import numpy as np
import pytest

import scenes

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# ---------------------------------------------------------------------------
# Appendix A known answers
# ---------------------------------------------------------------------------
def test_u8_readback_is_cvttsd2si_low_byte(oracle):
    # A.5: 1.8 -> 203, 1.2 -> 50, 2.4 -> 100; NaN / out of int32 range -> 0
    ctx = oracle.context(4, 1, False)
    ctx.set_pixel(0, 0, 1.8, 1.2, 2.4, 0)
    ctx.set_pixel(1, 0, -0.5, float("nan"), 1e12, 0)
    ctx.set_pixel(2, 0, 1.0, 0.999, -1e12, 0)
    u = ctx.get_buffer_as_uint8_numpy()[0]
    assert list(u[0]) == [203, 50, 100]
    assert list(u[1]) == [129, 0, 0]          # trunc(-127.5) = -127 -> 0x81
    assert list(u[2]) == [255, 254, 0]


def test_setpixel_overrun_rgb(oracle):
    # A.6: set_color(0.1,0.2,0.3,0.9) on RGB: column 0 of rows >= 1 reads [0.9, 0.2, 0.3]
    ctx = oracle.context(5, 4, False)
    ctx.set_color(0.1, 0.2, 0.3, 0.9)
    b = ctx.get_buffer_numpy()
    assert list(b[0, 0]) == [0.1, 0.2, 0.3]
    for y in range(1, 4):
        assert list(b[y, 0]) == [0.9, 0.2, 0.3]
    assert np.all(b[:, 1:] == np.array([0.1, 0.2, 0.3]))


def test_rect_coverage_edges(oracle):
    # A.7: x in [2.5, 6.5] covers {3,4,5}; [2, 6] covers {2,3,4,5}; y in [0,1] covers row 0
    ctx = oracle.context(10, 4, False)
    ctx.set_color(0, 0, 0, 0)
    ctx.draw_rect(2.5, 0, 4, 1, 1, 1, 1, 1)
    ctx.draw_rect(2, 2, 4, 1, 1, 1, 1, 1)
    b = ctx.get_buffer_numpy()[..., 0]
    assert list(np.nonzero(b[0])[0]) == [3, 4, 5]
    assert b[1].sum() == 0
    assert list(np.nonzero(b[2])[0]) == [2, 3, 4, 5]
    assert b[3].sum() == 0


def test_two_half_alpha_rects_rgba(oracle):
    # A.8: destination alpha is the source alpha, not composited
    ctx = oracle.context(4, 4, True)
    ctx.set_color(0, 0, 0, 0)
    ctx.draw_rect(0, 0, 3, 3, 1, 0, 0, 0.5)
    ctx.draw_rect(0, 0, 3, 3, 0, 1, 0, 0.5)
    assert list(ctx.get_buffer_numpy()[1, 1]) == [0.25, 0.5, 0.0, 0.5]


def test_isnotransform_signed_sum(oracle):
    # A.4: a pure rotation takes the fast path (transform ignored) for
    # draw_texture, while draw_rect honours it.
    tex = oracle.texture(np.full((8, 8, 4), 255, np.uint8))
    ctx = oracle.context(32, 32, True)
    ctx.set_color(0, 0, 0, 0)
    ctx.rotate(0.3)                 # sum = 2(cos 0.3 - 1) < 1e-5
    ctx.draw_texture(tex, 12, 12, 8, 8)
    b = ctx.get_buffer_numpy()[..., 3]
    ys, xs = np.nonzero(b)
    assert (ys.min(), ys.max(), xs.min(), xs.max()) == (12, 19, 12, 19) and len(ys) == 64
    ctx2 = oracle.context(32, 32, True)
    ctx2.set_color(0, 0, 0, 0)
    ctx2.rotate(0.3)
    ctx2.draw_rect(12, 12, 8, 8, 1, 1, 1, 1)
    b2 = ctx2.get_buffer_numpy()[..., 3]
    assert not np.array_equal(b2 > 0, b > 0)


def test_singular_inverse(oracle):
    # A.10: det == 0 -> inv_det = 1e9
    ctx = oracle.context(2, 2, False)
    ctx.set_transform(2, 0, 0, 0, 5, 7)
    inv = ctx.get_inverse_transform()
    assert inv == (0.0, -0.0, -0.0, 2e9, 0.0, -14 * 1e9)


def test_drawline_full_scan_under_singular_transform(oracle):
    # A.9: every pixel maps to (0,0) under a zero matrix; the polygon holds it
    ctx = oracle.context(6, 5, False)
    ctx.set_color(0, 0, 0, 0)
    ctx.set_transform(0, 0, 0, 0, 0, 0)
    ctx.draw_line(-1, -1, 1, 1, 2, 1, 1, 1, 1)
    assert np.all(ctx.get_buffer_numpy() == 1.0)


def test_sampler_never_reads_last_row_or_column(oracle):
    # A.3: clamp to [0, w-2] x [0, h-2]
    t = np.zeros((3, 3, 4), np.uint8)
    t[..., 3] = 255
    t[2, :, 0] = 255                # last row red
    t[:, 2, 1] = 255                # last column green
    tex = oracle.texture(t)
    ctx = oracle.context(3, 3, True)
    ctx.set_color(0, 0, 0, 0)
    ctx.draw_texture(tex, 0, 0, 3, 3)
    b = ctx.get_buffer_numpy()
    assert b[..., 0].max() == 0 and b[..., 1].max() == 0


def test_texture_u8_divides_by_255(oracle):
    t = np.arange(48, dtype=np.uint8).reshape(4, 3, 4) * 5
    t[..., 3] = 255
    tex = oracle.texture(t)
    ctx = oracle.context(3, 4, True)
    ctx.set_color(0, 0, 0, 0)
    ctx.draw_texture(tex, 0, 0, 3, 4)
    b = ctx.get_buffer_numpy()
    assert b[1, 1, 0] == t[1, 1, 0] / 255.0


# ---------------------------------------------------------------------------
# reference binding + fixtures
# ---------------------------------------------------------------------------
def _refbinding_names():
    return sorted(f[len("refbinding_"):-4] for f in os.listdir(GOLDEN) if f.startswith("refbinding_"))


@pytest.mark.parametrize("name", _refbinding_names())
def test_oracle_matches_reference_binding_fixture(oracle, name):
    fx = np.load(os.path.join(GOLDEN, f"refbinding_{name}.npz"))
    out = scenes.run_scene(name, oracle)
    for k in fx.files:
        assert scenes.bits_equal(out[k], fx[k]), scenes.first_mismatch(out[k], fx[k])


def test_oracle_matches_scene_fixtures(oracle):
    want = dict(line.split() for line in open(os.path.join(GOLDEN, "scenes.sha256")) if line.strip())
    for name in scenes.all_scenes():
        for k, v in scenes.run_scene(name, oracle).items():
            got = hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest()
            assert got == want[f"{name}/{k}"], f"{name}/{k}"


# ---------------------------------------------------------------------------
# triangle semantics — independent Python restatements
# ---------------------------------------------------------------------------
def py_point_in_polygon(x, y, pts):
    """cpp:822-845, evaluated in Python floats (IEEE double, same order)."""
    n = len(pts)
    j = n - 1
    res = False
    for i in range(n):
        if (pts[i][1] > y) != (pts[j][1] > y) and (
                x < (pts[j][0] - pts[i][0]) * (y - pts[i][1]) / (pts[j][1] - pts[i][1]) + pts[i][0]):
            res = not res
        j = i
    return res


def py_row_span(y, pts):
    """The GPU raster's rule (nr_tri.hip, phase b): the two straddling edges'
    crossings -> covered x in [ceil(min), ceil(max))."""
    c = []
    for i in range(3):
        j = (i + 2) % 3
        if (pts[i][1] > y) != (pts[j][1] > y):
            c.append((pts[j][0] - pts[i][0]) * (y - pts[i][1]) / (pts[j][1] - pts[i][1]) + pts[i][0])
    assert len(c) in (0, 2)
    if len(c) == 0:
        return 0, 0
    return math.ceil(min(c)), math.ceil(max(c))


def py_row_span_in(y, pts):
    """nr_tri.h row_span_in: for ymin <= y < ymax, the two edges at the vertex
    alone on its side of y, in pointInPolygon's (i, j) orientation."""
    b = [p[1] > y for p in pts]
    v1 = b[1] != b[0] and b[1] != b[2]
    v2 = b[2] != b[0] and b[2] != b[1]
    a = (2, 1) if v1 else (0, 2)
    bb = (2, 1) if v2 else (1, 0)
    c = [(pts[j][0] - pts[i][0]) * (y - pts[i][1]) / (pts[j][1] - pts[i][1]) + pts[i][0] for i, j in (a, bb)]
    return math.ceil(min(c)), math.ceil(max(c))


def py_row_span_slopes(y, pts):
    """nr_tri.h row_span_slopes: per-edge slopes, a division only when a
    crossing lies within eps of an integer (crossing_ceil)."""
    sx = [p[0] for p in pts]
    sy = [p[1] for p in pts]

    def slope(i, j):
        d = sy[j] - sy[i]
        return (sx[j] - sx[i]) / d if d != 0 else math.inf
    sl = [slope(0, 2), slope(1, 0), slope(2, 1)]
    b = [v > y for v in sy]
    v1 = b[1] != b[0] and b[1] != b[2]
    v2 = b[2] != b[0] and b[2] != b[1]
    ea, sa = ((2, 1), sl[2]) if v1 else ((0, 2), sl[0])
    eb, sb = ((2, 1), sl[2]) if v2 else ((1, 0), sl[1])
    ks, safe = [], True
    for (i, _), s_ in ((ea, sa), (eb, sb)):
        v = (y - sy[i]) * s_
        cc = v + sx[i]
        k = math.ceil(cc) if math.isfinite(cc) else 0
        eps = (abs(v) + abs(cc)) * 2.0 ** -50 + 2.0 ** -1000
        safe = safe and (cc - (k - 1.0) > eps) and (k - cc > eps)
        ks.append(k)
    if not safe:
        ks = [math.ceil((sx[j] - sx[i]) * (y - sy[i]) / (sy[j] - sy[i]) + sx[i]) for i, j in (ea, eb)]
    return min(ks), max(ks), safe


def py_row_span32(y, pts, x0, y0, wlim=64.0):
    """nr_tri.h row_span32 (f32 fast path of the row spans, restated with
    numpy float32): the two straddling edges chosen by the middle vertex's y,
    crossings relative to the tile origin in f32, and the error bound that
    decides whether the f32 ceil may be used.  Returns (xs, xe, ok)."""
    f = np.float32
    sx = [p[0] for p in pts]
    sy = [p[1] for p in pts]

    def slope(i, j):
        d = sy[j] - sy[i]
        return (sx[j] - sx[i]) / d if d != 0 else math.inf
    sl = [slope(0, 2), slope(1, 0), slope(2, 1)]
    a, b, c = sy
    imin = (2 if c < b else 1) if b < a else (2 if c < a else 0)
    imax = (2 if c >= b else 1) if b >= a else (2 if c >= a else 0)
    imid = 3 - imin - imax
    eid = lambda p, q: {2: 0, 1: 1, 3: 2}[p + q]

    def edge(k):
        with np.errstate(all="ignore"):
            xr, yr = sx[k] - x0, sy[k] - y0
            e_x, yhi = f(xr), f(yr)
            ylo = f(yr - float(yhi))
            s_ = f(sl[k])
            ce = f(abs(e_x) * f(2.0 ** -21) + abs(s_) * (abs(yhi) * f(2.0 ** -46) + f(abs(sy[k]) * 2.0 ** -51))
                   + f(abs(sx[k]) * 2.0 ** -51) + f(2.0 ** -23))
        return e_x, yhi, ylo, s_, ce

    L, T, B = edge(eid(imin, imax)), edge(eid(imin, imid)), edge(eid(imid, imax))
    E = T if y < sy[imid] else B
    rf = f(y - y0)
    ks, ok = [], True
    with np.errstate(all="ignore"):
        for (e_x, yhi, ylo, s_, ce) in (L, E):
            bb = (rf - yhi) - ylo
            v = bb * s_
            cc = v + e_x
            k = np.ceil(cc)
            d = k - cc
            eps = f(float(abs(cc)) * 2.0 ** -22 + float(f(float(abs(v)) * 2.0 ** -20 + float(ce))))
            ok = ok and bool(d > eps) and bool(f(1.0) - d > eps)
            ks.append(k)
    if not ok:
        return 0, 0, False
    lo, hi = min(ks), max(ks)
    return int(min(max(lo, 0.0), wlim)), int(min(max(hi, 0.0), wlim)), True


def _edge_case_triangles():
    g = scenes.rng(77)
    tris = [
        [(2, 2), (10, 2), (2, 10)], [(10, 2), (10, 10), (2, 10)], [(0.5, 0.5), (7.5, 3.5), (3.0, 9.0)],
        [(5, 5), (5, 5), (9, 9)], [(1, 1), (8, 1), (4.5, 1)], [(3.3, 7.0), (3.3, 1.0), (9.9, 4.0)],
        [(-3, -2), (6.5, 12), (11, -5)], [(4, 0), (4.000001, 9), (3.999999, 9)],
    ]
    for _ in range(200):
        c = g.uniform(0, 12, 2)
        tris.append([tuple(c + g.uniform(-6, 6, 2)) for _ in range(3)])
    for _ in range(100):   # integer / half-integer vertices hit pixel centres exactly
        tris.append([tuple(np.round(g.uniform(-2, 14, 2) * 2) / 2) for _ in range(3)])
    return tris


def test_row_span_rule_equals_point_in_polygon():
    for pts in _edge_case_triangles():
        for y in range(-3, 16):
            lo, hi = py_row_span(float(y), pts)
            for x in range(-4, 18):
                assert py_point_in_polygon(float(x), float(y), pts) == (lo <= x < hi), (pts, x, y)


def test_branchless_row_span_equals_row_span():
    for pts in _edge_case_triangles():
        ys = [p[1] for p in pts]
        for y in range(math.ceil(min(ys)), math.ceil(max(ys))):
            assert py_row_span_in(float(y), pts) == py_row_span(float(y), pts), (pts, y)


def test_slope_row_span_equals_row_span():
    g = scenes.rng(5)
    tris = list(_edge_case_triangles())
    for _ in range(3000):   # arbitrary geometry: the fast path is taken and must agree
        c = g.uniform(-50, 4000, 2)
        tris.append([tuple(c + g.normal(0, 6, 2)) for _ in range(3)])
    for _ in range(1000):   # integer / half-integer vertices: crossings land on integers
        c = g.integers(0, 60, 2)
        tris.append([tuple((c + g.integers(-8, 9, 2)) / g.choice([1, 2, 4])) for _ in range(3)])
    for _ in range(300):    # huge coordinates
        c = g.uniform(-1e9, 1e9, 2)
        tris.append([tuple(c + g.normal(0, 1e6, 2)) for _ in range(3)])
    fast = 0
    total = 0
    for pts in tris:
        ys = [p[1] for p in pts]
        lo, hi = math.ceil(min(ys)), math.ceil(max(ys))
        for y in range(lo, min(hi, lo + 40)):
            a, b, safe = py_row_span_slopes(float(y), pts)
            assert (a, b) == py_row_span(float(y), pts), (pts, y)
            fast += safe
            total += 1
    assert fast > total // 2


def test_oracle_triangle_coverage_equals_point_in_polygon(oracle):
    W, H = 14, 12
    for t, pts in enumerate(_edge_case_triangles()[:120]):
        ctx = oracle.context(W, H, False)
        ctx.set_color(0, 0, 0, 0)
        ctx.draw_triangles(np.array(pts, np.float64).reshape(1, 6), np.array([[1.0, 1, 1, 1]]))
        got = ctx.get_buffer_numpy()[..., 0] == 1.0
        want = np.zeros((H, W), bool)
        e1x, e1y = pts[1][0] - pts[0][0], pts[1][1] - pts[0][1]
        e2x, e2y = pts[2][0] - pts[0][0], pts[2][1] - pts[0][1]
        if e1x * e2y - e2x * e1y != 0:
            for y in range(H):
                for x in range(W):
                    want[y, x] = py_point_in_polygon(float(x), float(y), pts)
        assert np.array_equal(got, want), (t, pts)
        assert ctx.last_fragment_count() == want.sum()


def test_oracle_gouraud_depth_formula(oracle):
    pts = [(1.25, 0.5), (9.5, 2.0), (3.0, 8.75)]
    col = [0.1, 0.2, 0.3, 1.0, 0.9, 0.5, 0.0, 1.0, 0.4, 0.8, 0.6, 1.0]
    zv = [0.2, 0.7, 0.45]
    ctx = oracle.context(12, 10, False)
    ctx.set_color(0, 0, 0, 0)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    ctx.draw_triangles(np.array(pts, np.float64).reshape(1, 6), np.array([col]), z=np.array([zv]))
    b, d = ctx.get_buffer_numpy(), ctx.get_depth_buffer()
    e1x, e1y = pts[1][0] - pts[0][0], pts[1][1] - pts[0][1]
    e2x, e2y = pts[2][0] - pts[0][0], pts[2][1] - pts[0][1]
    inv = 1.0 / (e1x * e2y - e2x * e1y)
    n = 0
    for y in range(10):
        for x in range(12):
            if not py_point_in_polygon(float(x), float(y), pts):
                assert d[y, x] == 0xFFFFFFFF
                continue
            dx, dy = x - pts[0][0], y - pts[0][1]
            w1 = (dx * e2y - e2x * dy) * inv
            w2 = (e1x * dy - dx * e1y) * inv
            z = zv[0] + (zv[1] - zv[0]) * w1 + (zv[2] - zv[0]) * w2
            zq = 0 if not z > 0 else (0xFFFFFFFF if z >= 1 else int(z * 4294967295.0))
            assert d[y, x] == zq
            for k in range(3):
                c = col[k] + (col[4 + k] - col[k]) * w1 + (col[8 + k] - col[k]) * w2
                assert b[y, x, k] == c
            n += 1
    assert n > 10


def test_oracle_depth_is_order_independent_min(oracle):
    # LESS + write: the final depth is min(clear, min zq) whatever the order
    xy, z, c = scenes.triangle_soup(300, 40, 30, 8, seed=3)
    perm = scenes.rng(4).permutation(300)
    outs = []
    for order in (np.arange(300), perm):
        ctx = oracle.context(40, 30, False)
        ctx.set_color(0, 0, 0, 0)
        ctx.set_depth_state(True, True)
        ctx.clear_depth()
        ctx.draw_triangles(xy[order], c[order], z=z[order])
        outs.append(ctx.get_depth_buffer())
    assert np.array_equal(outs[0], outs[1])
    assert (outs[0] != 0xFFFFFFFF).sum() > 500


def test_sphere_mesh_shape():
    xy, z, c = scenes.sphere_mesh(64, 48, 10, 20)
    assert xy.shape == (400, 6) and z.shape == (400, 3) and c.shape == (400, 12)
    assert np.all((z > 0) & (z < 1))


def _py_hit_pixel(seed, t, x, y):
    """Independent restatement of cpp:1318-1410 (Python floats are the same
    IEEE doubles and libm): GetMilthmHitEffectPixel."""
    fract = lambda v: v - math.floor(v)
    rand = lambda nx, ny: fract(math.sin(nx * 12.9898 + ny * 78.233) * 43758.5453)
    mix = lambda a, b, k: a + (b - a) * k

    def noise(px, py):
        ix, iy = math.floor(px), math.floor(py)
        ux, uy = fract(px), fract(py)
        a, b = rand(ix, iy), rand(ix + 1.0, iy + 0.0)
        c, d = rand(ix + 0.0, iy + 1.0), rand(ix + 1.0, iy + 1.0)
        sx, sy = ux * ux * (3.0 - 2.0 * ux), uy * uy * (3.0 - 2.0 * uy)
        return mix(mix(a, b, sx), mix(c, d, sx), sy)

    cx, cy = x - 0.5, y - 0.5
    radius = math.sqrt(cx * cx + cy * cy) * 50.0
    angle = abs(math.atan2(cy, cx))          # std::abs(double) in the reference build
    if y > 0.5:
        angle += math.sin(angle) * 2.0
    px, py = radius + seed * 100.0, angle + seed * 100.0
    n = 0.0
    n += noise(px, py) * 0.7
    n += noise(px * 2.0, py * 2.0) * 0.3
    n += noise(px * 4.0, py * 4.0) * 0.1
    return 0.0 if n < t else 1.0


@pytest.mark.parametrize("w,h", [(9, 13), (16, 16)])
def test_oracle_hit_effect_texture(w, h):
    """CreateMilthmHitEffectTexture (cpp:1416-1438): colour constant, alpha =
    pixel(i/w, j/h) * mask alpha, texel (i, j) stored at (i*h + j)*4 and the
    mask read at that same index (column-major, cpp:1413-1432)."""
    mask = scenes.hit_mask(w, h)
    seed, t = 0.37, 0.45
    out = scenes.oracle_hit_effect(mask, seed, t).reshape(-1)
    flat_mask = (mask.astype(np.float64) / 255.0).reshape(-1)
    for i in range(w):
        for j in range(h):
            q = (i * h + j) * 4
            want = _py_hit_pixel(seed, t, i / w, j / h) * flat_mask[q + 3]
            assert out[q + 3] == want, (i, j)
            assert out[q] == 0x96 / 0xff and out[q + 1] == 0x90 / 0xff and out[q + 2] == 0xfd / 0xff
    assert 0 < np.count_nonzero(out[3::4]) < w * h   # both sides of the threshold occur


def test_oracle_hit_effect_needs_alpha():
    lib = scenes._OracleLib.get()
    rgb = np.zeros((4, 4, 3), dtype=np.uint8)
    m = lib.CreateTextureUInt8(4, 4, False, rgb.ctypes.data_as(scenes.ctypes.c_void_p))
    assert not lib.CreateMilthmHitEffectTexture(m, 0.1, 0.5, 1.0, 1.0, 1.0)   # NULL (cpp:1418)


def test_yuv420p_restatement_known_values():
    """BT.601 limited range with this converter's truncating shift: black ->
    (16, 128, 128); white -> (234, 128, 128) and pure red -> (81, 90, 239),
    one below the nominal 235 / 240 where the product sum is just under the
    next integer (the fast path truncates instead of rounding)."""
    for rgb, want in (((0, 0, 0), (16, 128, 128)), ((255, 255, 255), (234, 128, 128)), ((255, 0, 0), (81, 90, 239))):
        img = np.zeros((2, 2, 3), dtype=np.uint8)
        img[...] = rgb
        out = scenes.yuv420p(img)
        assert tuple(int(v) for v in (out[0], out[4], out[5])) == want


def test_f32_row_span_equals_row_span():
    """row_span32 (the f32 fast path of k_vis's row spans): whenever its error
    bound accepts the f32 crossings, the span relative to the tile origin and
    clamped to the tile equals the exact rule's (integer-aligned vertices,
    steep edges and huge coordinates included: the relative coordinates keep
    the bound small even at 1e9); on arbitrary geometry it accepts > 99.5 %
    of the rows."""
    g = scenes.rng(6)
    kinds = [("edge", t) for t in _edge_case_triangles()]
    for _ in range(3000):   # C3-like slivers and C2-like small triangles at 4K coordinates
        c = g.uniform(-50, 4000, 2)
        kinds.append(("arb", [tuple(c + g.normal(0, g.choice([0.7, 3, 12]), 2)) for _ in range(3)]))
    for _ in range(600):    # steep / near-horizontal edges
        c = g.uniform(0, 2000, 2)
        kinds.append(("steep", [tuple(c), tuple(c + (g.normal(0, 30), g.normal(0, 0.01))), tuple(c + g.normal(0, 5, 2))]))
    for _ in range(800):    # integer / half-integer vertices: crossings land on integers
        c = g.integers(0, 60, 2)
        kinds.append(("int", [tuple((c + g.integers(-8, 9, 2)) / g.choice([1, 2, 4])) for _ in range(3)]))
    for _ in range(200):    # huge coordinates
        c = g.uniform(-1e9, 1e9, 2)
        kinds.append(("huge", [tuple(c + g.normal(0, 1e6, 2)) for _ in range(3)]))
    acc, total = {}, {}
    for kind, pts in kinds:
        ys = [p[1] for p in pts]
        if len({p[1] for p in pts}) == 1:
            continue
        lo, hi = math.ceil(min(ys)), math.ceil(max(ys))
        for y in range(lo, min(hi, lo + 40)):
            xlo, xhi = py_row_span(float(y), pts)
            if (xlo, xhi) == (0, 0):
                continue
            ty = math.floor(y / 32) * 32
            for x0 in {math.floor(min(p[0] for p in pts) / 64) * 64, math.floor(xlo / 64) * 64}:
                xs, xe, ok = py_row_span32(float(y), pts, float(x0), float(ty))
                total[kind] = total.get(kind, 0) + 1
                if not ok:
                    continue
                acc[kind] = acc.get(kind, 0) + 1
                want = (min(max(xlo - x0, 0), 64), min(max(xhi - x0, 0), 64))
                assert (xs, xe) == want, (kind, pts, y, x0, (xs, xe), want)
    assert acc["arb"] > 0.995 * total["arb"], (acc, total)
