"""Depth quantisation at the edges of its domain: the rasters convert z to u32
with one saturating hardware conversion (nr_quantize_depth_hw: v_cvt_u32_f64
truncates, clamps to [0, 0xFFFFFFFF] and maps NaN to 0), which must equal the
oracle's clamp (z <= 0 or NaN -> 0, z >= 1 -> 0xFFFFFFFF, else (u32)(z *
4294967295.0)) bit for bit.  Vertex depths NaN, +-inf, +-1e300, just below
and above 0 and 1, and values whose product lands next to an integer; drawn
through the order-free raster (LESS + write) and the ordered raster (LESS
without write: the depth-pass proof does not apply to non-finite depths)."""
import numpy as np
import pytest

import scenes

pytestmark = pytest.mark.gpu

EDGE_Z = [float("nan"), float("inf"), -float("inf"), 1e300, -1e300, 0.0, -0.0, 5e-324, -5e-324,
          1.0, np.nextafter(1.0, 0.0), np.nextafter(1.0, 2.0), 0.5, 1.0 / 4294967295.0,
          np.nextafter(1.0 / 4294967295.0, 0.0), 2.0 / 4294967295.0, 0.25 + 1e-17, 0.75]


def _scene(W, H, seed):
    rng = np.random.default_rng(seed)
    n = 240
    c = np.stack([rng.uniform(0, W, n), rng.uniform(0, H, n)], axis=1)
    xy = (c[:, None, :] + rng.uniform(-40, 40, size=(n, 3, 2))).reshape(n, 6)
    z = rng.choice(np.array(EDGE_Z), size=(n, 3))
    z[::3] = rng.uniform(-0.2, 1.2, size=z[::3].shape)   # a third ordinary, for contrast
    z[1::7] = z[1::7, :1]                                  # constant-depth triangles (one edge value each)
    col = rng.uniform(0, 1, size=(n, 12))
    col[:, 3::4] = 1.0
    return xy, z, col


@pytest.mark.parametrize("mode", ["less_write", "less_nowrite", "blended"])
def test_depth_edge_values_match_oracle(gpu, oracle, mode):
    W, H = 200, 140
    xy, z, col = _scene(W, H, 11)
    outs = {}
    for fac in (gpu, oracle):
        ctx = fac.context(W, H, False)
        ctx.set_color(0.2, 0.2, 0.2, 0.2)
        ctx.set_depth_state(True, True)
        ctx.clear_depth(0x80000000)
        # a written layer first (ordinary depths), then the edge-value batch
        ctx.draw_triangles(xy[::3], col[::3], z=z[::3])
        if mode == "less_write":
            ctx.draw_triangles(xy, col, z=z)
        elif mode == "less_nowrite":
            ctx.set_depth_state(True, False)
            ctx.draw_triangles(xy, col, z=z)
        else:
            cb = col.copy()
            cb[:, 3::4] = 0.5
            ctx.set_depth_state(True, False)
            ctx.draw_triangles(xy, cb, z=z)
        outs[fac.name] = (ctx.get_buffer_numpy(), ctx.get_depth_buffer())
    (gf, gd), (of, od) = outs["gpu"], outs["oracle"]
    assert scenes.bits_equal(gf, of), scenes.first_mismatch(gf, of)
    assert np.array_equal(gd, od), scenes.first_mismatch(gd, od)
