"""GPU parity: the HIP library (through its Pybind mirror) against the CPU
oracle on the same seeded inputs, bit for bit (f64 framebuffer, u8 readback,
u32 depth), at fixture sizes and at BASELINE.json's full sizes."""
import ctypes
import os

import numpy as np
import pytest

import scenes

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def assert_same(a: dict, b: dict, what=""):
    assert set(a) == set(b), (what, set(a) ^ set(b))
    for k in a:
        assert scenes.bits_equal(a[k], b[k]), f"{what}/{k}: {scenes.first_mismatch(a[k], b[k])}"


@pytest.mark.parametrize("name", sorted(scenes.all_scenes()))
def test_scene_parity(gpu, oracle, golden, name):
    g = scenes.run_scene(name, gpu)
    o = scenes.run_scene(name, oracle)
    assert_same(g, o, name)
    for k, v in g.items():
        assert scenes.bits_equal(v, golden[f"{name}/{k}"]), f"{name}/{k} vs golden"


def _c1(fac, rotated):
    img = np.load(os.path.join(GOLDEN, "image_png_rgba.npy"))
    ctx = fac.context(256, 256, True)
    ctx.set_color(0, 0, 0, 0)
    tex = fac.texture(img)
    if rotated:
        ctx.translate(128, 128)
        ctx.rotate(0.3)
        ctx.translate(-128, -128)
    ctx.draw_texture(tex, 64, 64, 128, 128)
    return {"f64": ctx.get_buffer_numpy(), "u8": ctx.get_buffer_as_uint8_numpy()}


@pytest.mark.parametrize("rotated", [False, True])
def test_c1_textured_quad(gpu, oracle, rotated):
    assert_same(_c1(gpu, rotated), _c1(oracle, rotated), f"C1 rotated={rotated}")


def _tri_frame(fac, W, H, xy, z, c, depth=True, write=True, alpha=False, clear=0.0):
    ctx = fac.context(W, H, alpha)
    ctx.set_color(clear, clear, clear, clear)
    ctx.set_depth_state(depth, write)
    ctx.clear_depth()
    ctx.draw_triangles(xy, c, z=z)
    out = {"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()}
    return out, ctx


def test_c2_flat_depth_1080p(gpu, oracle):
    xy, z, c = scenes.triangle_soup(10000, 1920, 1080, 32, seed=1234)
    g, gctx = _tri_frame(gpu, 1920, 1080, xy, z, c)
    o, octx = _tri_frame(oracle, 1920, 1080, xy, z, c)
    assert_same(g, o, "C2")


@pytest.mark.parametrize("mode", [1, 2])
def test_vis_variants_match_oracle(gpu, oracle, mode):
    """Both k_vis variants (1: wave-cooperative pass for large triangles, 2:
    lane per triangle only) on a soup mixing large and small triangles, in
    every depth mode, RGB and RGBA."""
    big = scenes.triangle_soup(300, 400, 300, 90, seed=41, gouraud=True)
    small = scenes.triangle_soup(3000, 400, 300, 4, seed=42, gouraud=True)
    xy = np.concatenate([big[0], small[0]]); z = np.concatenate([big[1], small[1]])
    c = np.concatenate([big[2], small[2]])
    perm = np.random.Generator(np.random.PCG64(43)).permutation(len(xy))
    xy, z, c = xy[perm], z[perm], c[perm]
    for depth, write in ((True, True), (True, False), (False, True)):
        for alpha in (False, True):
            outs = []
            for fac in (gpu, oracle):
                ctx = fac.context(400, 300, alpha)
                if fac is gpu:
                    ctx.set_coop_raster(mode)
                ctx.set_color(0.25, 0.25, 0.25, 0.25)
                ctx.set_depth_state(depth, write)
                ctx.clear_depth()
                ctx.draw_triangles(xy, c, z=z)
                outs.append({"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()})
            assert_same(outs[0], outs[1], f"mode={mode} depth={depth} write={write} alpha={alpha}")


def test_c3_gouraud_depth_4k(gpu, oracle):
    """C3 at full size (the tiled k_vis) against the oracle frame."""
    xy, z, c = scenes.sphere_mesh(3840, 2160, 500, 1000)
    o, _ = _tri_frame(oracle, 3840, 2160, xy, z, c)
    g, ctx = _tri_frame(gpu, 3840, 2160, xy, z, c)
    assert ctx.last_raster_path() == "order-free"
    assert_same(g, o, "C3 order-free")


def test_c5_blend_overdraw_reduced(gpu, oracle):
    # C5 shape (back-to-front, a in [0.2, 0.8], Z test on, write off) at 1/10
    # of the triangle count so the oracle finishes in seconds.
    xy, z, c = scenes.triangle_soup(5000, 1920, 1080, 256, seed=1234, alpha=(0.2, 0.8))
    order = np.argsort(-z.mean(axis=1), kind="stable")
    xy, z, c = xy[order], z[order], c[order]
    g, _ = _tri_frame(gpu, 1920, 1080, xy, z, c, write=False)
    o, _ = _tri_frame(oracle, 1920, 1080, xy, z, c, write=False)
    assert_same(g, o, "C5/10")


def _blend_chunks_frame(fac, W, H, alpha, test):
    """The ordered raster's blend-only chunk loop and its neighbours: flat
    translucent triangles in 64-triangle chunks where some chunks hold an
    opaque (a = 1) triangle (those chunks take the general loop), a right-edge
    tile narrower than 64 columns, spans ending at the tile edge, a colour
    transform, and Z test on (write off) or off."""
    ctx = fac.context(W, H, alpha)
    ctx.set_color(0.3, 0.6, 0.1, 0.7)
    ctx.set_depth_state(test, False)
    ctx.clear_depth()
    ctx.set_color_transform(0.9, 1.0, 0.8, 0.95)
    xy, z, c = scenes.triangle_soup(1500, W, H, 120.0, seed=4242, alpha=(0.2, 0.8))
    c = c.copy()
    c[::97, 3] = 1.0                      # a few opaque triangles: their chunks take the general loop
    xy[::53, 0::2] = np.clip(xy[::53, 0::2], W - 30, W + 30)   # triangles over the narrow right-edge tile
    ctx.draw_triangles(xy, c, z=z)
    return {"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer(), "u8": ctx.get_buffer_as_uint8_numpy()}


@pytest.mark.parametrize("alpha", [False, True])
@pytest.mark.parametrize("test", [False, True])
def test_blend_only_chunks_match_oracle(gpu, oracle, alpha, test):
    W, H = 360, 200   # 6 tile columns, the last 40 wide; 7 tile rows, the last 8 high
    assert_same(_blend_chunks_frame(gpu, W, H, alpha, test), _blend_chunks_frame(oracle, W, H, alpha, test),
                f"blend chunks alpha={alpha} test={test}")


def _zpass_edges_frame(fac, W, H):
    """Z test without write over a non-uniform depth layer, with depths at the
    edge of the ordered raster's per-triangle pass proof (zpass_all): a
    written layer at z = 0.5 (+ per-triangle offsets), then blended batches
    whose depths sit 1e-12 .. 1e-6 below / at / above it, near-1 depths over
    the cleared 0xFFFFFFFF buffer, slivers and huge coordinates."""
    g = np.random.default_rng(77)
    ctx = fac.context(W, H, False)
    ctx.set_color(0.25, 0.25, 0.25, 0.25)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    xy, _, c = scenes.triangle_soup(60, W, H, 60.0, seed=5)
    z = 0.5 + g.choice([0.0, 1e-9, -1e-9, 3e-7], size=(60, 1)) + np.zeros((60, 3))
    ctx.draw_triangles(xy, c, z=z)   # opaque layer, Z written
    ctx.set_depth_state(True, False)
    for k, off in enumerate([-1e-6, -1e-9, -1e-12, 0.0, 1e-12, 1e-9]):
        xy, _, c = scenes.triangle_soup(80, W, H, 90.0, seed=100 + k, alpha=(0.2, 0.8))
        z = np.full((80, 3), 0.5 + off) + g.uniform(0, 1e-10, size=(80, 3)) * (k % 2)
        ctx.draw_triangles(xy, c, z=z)
    # over the cleared buffer only: depths at and just below 1
    ctx.clear_depth()
    xy, _, c = scenes.triangle_soup(80, W, H, 90.0, seed=300, alpha=(0.2, 0.8))
    z = 1.0 - g.choice([0.0, 1e-15, 1e-12, 1e-9, 1e-7], size=(80, 3))
    ctx.draw_triangles(xy, c, z=z)
    # slivers (ill-conditioned: the proof must decline them) and huge coordinates
    sl = np.array([[10, 10, 250, 11, 130, 10.5], [5, 120, 6, 5, 5.5, 60], [0, 0, 1e6, 1, -1e6, 2],
                   [-3e7, 64, 3e7, 65, 0, -3e7]], np.float64)
    cs = np.tile(np.array([[0.9, 0.1, 0.3, 0.5]]), (len(sl), 1))
    ctx.draw_triangles(sl, cs, z=np.full((len(sl), 3), 0.999999))
    return {"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer(), "u8": ctx.get_buffer_as_uint8_numpy()}


def test_depth_pass_proof_edges(gpu, oracle):
    assert_same(_zpass_edges_frame(gpu, 256, 160), _zpass_edges_frame(oracle, 256, 160), "zpass edges")


@pytest.mark.slow
def test_c5_blend_overdraw_full(gpu, oracle):
    """C5 at its full size (BASELINE configs[4]: 50k large alpha-blended
    triangles back to front, 1080p; ~1 G blended fragments, ~12 s on the
    oracle), bit-exact f64 and depth."""
    xy, z, c = scenes.triangle_soup(50000, 1920, 1080, 256, seed=1234, alpha=(0.2, 0.8))
    order = np.argsort(-z.mean(axis=1), kind="stable")
    xy, z, c = xy[order], z[order], c[order]
    g, _ = _tri_frame(gpu, 1920, 1080, xy, z, c, write=False)
    o, _ = _tri_frame(oracle, 1920, 1080, xy, z, c, write=False)
    assert_same(g, o, "C5")


def test_fragment_counter_matches_oracle(gpu, oracle):
    xy, z, c = scenes.triangle_soup(3000, 640, 480, 20, seed=8, gouraud=True)
    ctx = gpu.context(640, 480, False)
    ctx.set_color(0, 0, 0, 0)
    ctx.set_fragment_counting(True)
    ctx.draw_triangles(xy, c, z=z)
    octx = oracle.context(640, 480, False)
    octx.set_color(0, 0, 0, 0)
    octx.draw_triangles(xy, c, z=z)
    assert ctx.get_fragment_count() == octx.last_fragment_count() > 0


def test_triangle_buffer_equals_host_arrays(gpu):
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    xy, z, c = scenes.triangle_soup(5000, 500, 300, 15, seed=9, gouraud=True)
    a, _ = _tri_frame(gpu, 500, 300, xy, z, c)
    ctx = gpu.context(500, 300, False)
    ctx.set_color(0, 0, 0, 0)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    buf = R.TriangleBuffer(xy, c, z=z)
    ctx.draw_triangle_buffer(buf)
    assert_same(a, {"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()}, "buffer")


@pytest.mark.parametrize("gouraud", [False, True])
def test_ordered_tile_list_over_sort_cap(gpu, oracle, gouraud):
    """A blended batch (ordered raster) with more triangles in one tile than
    its per-tile LDS sort holds (ORD_SORT_CAP = 8192): the plan kernel flags it
    and the batch takes the global-sort path -- at once for host arrays (sized
    in the call), through the deferred re-run for a TriangleBuffer (its raster
    was a no-op).  Flat with no Z test, Gouraud with the Z test on and write
    off.  Same frame as the oracle either way."""
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    W, H = 150, 70
    xy, z, c = scenes.triangle_soup(9000, 56, 26, 4.0, seed=71, gouraud=gouraud, alpha=(0.3, 0.7))
    want, _ = _tri_frame(oracle, W, H, xy, z, c, depth=gouraud, write=False, alpha=True, clear=0.25)
    got, _ = _tri_frame(gpu, W, H, xy, z, c, depth=gouraud, write=False, alpha=True, clear=0.25)
    assert_same(got, want, "host arrays")
    ctx = gpu.context(W, H, True)
    for _ in range(2):   # (the second draw reuses the binning set of the first)
        ctx.set_color(0.25, 0.25, 0.25, 0.25)
        ctx.set_depth_state(gouraud, False)
        ctx.clear_depth()
        ctx.draw_triangle_buffer(R.TriangleBuffer(xy, c, z=z, gouraud=gouraud))
        assert_same({"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()}, want, "TriangleBuffer")


def _overcap_then_clear_depth(fac, W, H, over, opaque_a, opaque_c, buffer):
    """An opaque batch (writes depth), then a blended batch with a tile list
    over ORD_SORT_CAP (a TriangleBuffer: its binned raster is a no-op that the
    next call re-runs), then ClearDepth -- which only marks the clear pending,
    without settling -- and another depth-writing batch, which must see the
    cleared depth: the deferred re-run must not consume the later clear."""
    ctx = fac.context(W, H, True)
    ctx.set_color(0.25, 0.25, 0.25, 0.25)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    ctx.draw_triangles(opaque_a[0], opaque_a[2], z=opaque_a[1])
    ctx.set_depth_state(True, False)
    if buffer:
        from libnativecpurenderer_amd import libNativeCPURendererPybind as R
        ctx.draw_triangle_buffer(R.TriangleBuffer(over[0], over[2], z=over[1], gouraud=True))
    else:
        ctx.draw_triangles(over[0], over[2], z=over[1])
    ctx.clear_depth()
    ctx.set_depth_state(True, True)
    ctx.draw_triangles(opaque_c[0], opaque_c[2], z=opaque_c[1])
    return {"f64": ctx.get_buffer_numpy(), "u8": ctx.get_buffer_as_uint8_numpy(), "depth": ctx.get_depth_buffer()}


def test_overcap_rerun_keeps_later_depth_clear(gpu, oracle):
    """the settle-time re-run of an over-cap ordered batch
    used to end with the flag bookkeeping of a fresh draw (pendDepth /
    pendColor / frameU8Valid overwritten from the old batch's snapshot)."""
    W, H = 150, 70
    over = scenes.triangle_soup(9000, 56, 26, 4.0, seed=71, gouraud=True, alpha=(0.3, 0.7))
    a = scenes.triangle_soup(200, W, H, 20.0, seed=72, gouraud=True)
    c = scenes.triangle_soup(200, W, H, 20.0, seed=73, gouraud=True)
    want = _overcap_then_clear_depth(oracle, W, H, over, a, c, buffer=False)
    got = _overcap_then_clear_depth(gpu, W, H, over, a, c, buffer=True)
    assert_same(got, want, "over-cap re-run, then ClearDepth")


def test_overcap_rerun_keeps_frame_output_stale_flag(gpu, oracle):
    """The same re-run followed by a non-uniform SetColor (which marks the u8
    frame mirror stale and then settles): the gathered u8 frame must be the
    one of the new colours, not the mirror the re-run wrote."""
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    W, H = 150, 70
    over = scenes.triangle_soup(9000, 56, 26, 4.0, seed=71, gouraud=False, alpha=(0.3, 0.7))
    ctx = gpu.context(W, H, False)
    ctx.set_color(0.5, 0.5, 0.5, 0.5)
    ctx.gather_frame_u8()   # the frame output is produced by the rasters from now on
    ctx.set_color(0.25, 0.25, 0.25, 0.25)
    ctx.set_depth_state(False, False)
    ctx.draw_triangle_buffer(R.TriangleBuffer(over[0], over[2], z=over[1], gouraud=False))
    ctx.set_color(0.1, 0.2, 0.3, 0.9)
    ctx.gather_frame_u8()
    got = ctx.get_frame_u8()
    octx = oracle.context(W, H, False)
    octx.set_color(0.1, 0.2, 0.3, 0.9)
    want = octx.get_buffer_as_uint8_numpy()
    assert scenes.bits_equal(got.reshape(want.shape), want), scenes.first_mismatch(got.reshape(want.shape), want)


def _grid_growth_frame(fac, W, H):
    """A tiny opaque batch, then one with ~20x its work items, in one context:
    the second batch's k_vis grid is estimated from the first (last items
    + 25 %, >= 1024 workgroups), far fewer than its items, so the grid-stride
    loop must cover the rest; then a smaller batch again (grid > items)."""
    ctx = fac.context(W, H, False)
    ctx.set_color(0.5, 0.5, 0.5, 0.5)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    for n, spread, seed in [(40, 6.0, 21), (1200000, 2.0, 22), (300, 40.0, 23)]:
        xy, z, c = scenes.triangle_soup(n, W, H, spread, seed=seed, gouraud=True)
        ctx.draw_triangles(xy, c, z=z)
    return {"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()}


def test_kvis_grid_smaller_than_items(gpu, oracle):
    # 1024x1024: 512 tiles, so the first batch's 512 items give a grid of 1024
    # workgroups; the 1.2M-triangle batch puts ~2300 pairs in every tile
    # (3 slices each): ~1500 items for those 1024 workgroups
    assert_same(_grid_growth_frame(gpu, 1024, 1024), _grid_growth_frame(oracle, 1024, 1024), "grid growth")


def test_triangle_buffer_repeat_draws_sized_from_known_totals(gpu):
    """A TriangleBuffer drawn again under the binning key (transform, frame,
    shard) of its last validated draw is sized from the recorded totals and
    not validated on the host.  Alternate keys (transforms, sizes, shards) and
    repeats: every frame equals the same draw from host arrays (validated)."""
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    xy, z, c = scenes.triangle_soup(6000, 420, 300, 16, seed=71, gouraud=True)
    buf = R.TriangleBuffer(xy, c, z=z)
    states = [((0, 0), 420, 300, None), ((0, 0), 420, 300, None), ((7.5, -3.25), 420, 300, None),
              ((0, 0), 420, 300, None), ((0, 0), 400, 300, None), ((0, 0), 420, 300, (3, 1)),
              ((0, 0), 420, 300, (3, 1)), ((0, 0), 420, 300, None), ((7.5, -3.25), 420, 300, None)]
    ctxs = {}
    for i, (t, W, H, shard) in enumerate(states):
        outs = []
        for use_buf in (True, False):
            key = (W, H, use_buf)
            if key not in ctxs:
                ctxs[key] = gpu.context(W, H, False)
            ctx = ctxs[key]
            if shard is None:
                ctx.set_shard(1, 0)
            else:
                ctx.set_shard(*shard)
            ctx.set_transform(1, 0, 0, 1, *t)
            ctx.set_color(0.1, 0.1, 0.1, 0.1)
            ctx.set_depth_state(True, True)
            ctx.clear_depth()
            if use_buf:
                ctx.draw_triangle_buffer(buf)
            else:
                ctx.draw_triangles(xy, c, z=z)
            ctx.gather_frame_u8()
            outs.append({"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer(), "u8": ctx.get_frame_u8()})
        assert_same(outs[0], outs[1], f"repeat {i}")


@pytest.mark.parametrize("misalign", [False, True])
def test_device_arrays_match_oracle(gpu, oracle, misalign):
    """DrawTrianglesDevice on torch HBM tensors, 16-byte aligned or not
    (misaligned arrays are re-staged: the kernels load 16-byte vectors)."""
    import torch
    xy, z, c = scenes.triangle_soup(5000, 500, 300, 15, seed=19, gouraud=True)
    a, _ = _tri_frame(oracle, 500, 300, xy, z, c)
    o = 1 if misalign else 0

    def dev(arr):
        flat = np.ascontiguousarray(arr, np.float64).ravel()
        t = torch.zeros(flat.size + o, dtype=torch.float64, device="cuda")
        t[o:] = torch.from_numpy(flat).to("cuda")
        return t[o:]
    dxy, dz, dc = dev(xy), dev(z), dev(c)
    assert (dxy.data_ptr() % 16 != 0) == misalign
    torch.cuda.synchronize()
    ctx = gpu.context(500, 300, False)
    ctx.set_color(0, 0, 0, 0)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    ctx.draw_triangles_device(dxy, dc, len(xy), z=dz, gouraud=True)
    assert_same(a, {"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()}, "device")


def test_c3_order_independent_depth_full_size(gpu):
    """Size-independent property at full C3 size: with LESS + write the depth
    buffer is min(clear, min zq) whatever the submission order."""
    xy, z, c = scenes.sphere_mesh(3840, 2160, 500, 1000)
    perm = scenes.rng(3).permutation(len(xy))
    a, _ = _tri_frame(gpu, 3840, 2160, xy, z, c)
    b, _ = _tri_frame(gpu, 3840, 2160, xy[perm], z[perm], c[perm])
    assert np.array_equal(a["depth"], b["depth"])
    assert (a["depth"] != 0xFFFFFFFF).sum() > 3_000_000


def test_repeat_frames_are_deterministic(gpu):
    xy, z, c = scenes.triangle_soup(20000, 1280, 720, 40, seed=10, alpha=(0.3, 1.0))
    outs = [_tri_frame(gpu, 1280, 720, xy, z, c, write=False)[0] for _ in range(2)]
    assert_same(outs[0], outs[1], "repeat")


def test_empty_and_offscreen_batches(gpu, oracle):
    xy = np.array([[-50, -50, -40, -45, -45, -30], [5000, 10, 5100, 20, 5050, 40]], np.float64)
    c = np.ones((2, 4))
    for n in (0, 2):
        g, _ = _tri_frame(gpu, 64, 64, xy[:n], None, c[:n], clear=0.5)
        o, _ = _tri_frame(oracle, 64, 64, xy[:n], None, c[:n], clear=0.5)
        assert_same(g, o, f"empty n={n}")


def test_resize_and_reuse(gpu, oracle):
    outs = []
    for fac in (gpu, oracle):
        ctx = fac.context(50, 40, False)
        ctx.set_color(0, 0, 0, 0)
        ctx.draw_rect(3, 3, 20, 20, 1, 0, 0, 1)
        ctx.resize(70, 33)
        ctx.set_color(0.3, 0.3, 0.3, 0.3)
        xy, z, c = scenes.triangle_soup(300, 70, 33, 8, seed=12)
        ctx.set_depth_state(True, True)
        ctx.clear_depth()
        ctx.draw_triangles(xy, c, z=z)
        outs.append({"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()})
    assert_same(outs[0], outs[1], "resize")


@pytest.mark.parametrize("mode", ["depth_write", "depth_nowrite", "nodepth"])
@pytest.mark.parametrize("gouraud", [False, True])
def test_order_free_equals_ordered(gpu, mode, gouraud):
    """The order-free raster (opaque batches) and the ordered raster agree bit
    for bit, and the opaque batch really takes the order-free path."""
    xy, z, c = scenes.triangle_soup(4000, 700, 500, 25, seed=31, gouraud=gouraud)
    outs = []
    for force in (False, True):
        ctx = gpu.context(700, 500, True)
        ctx.set_force_ordered_raster(force)
        ctx.set_color(0.25, 0.25, 0.25, 0.25)
        ctx.set_depth_state(mode != "nodepth", mode == "depth_write")
        ctx.clear_depth(0xF0000000)
        ctx.draw_triangles(xy, c, z=z)
        assert ctx.last_raster_path() == ("ordered" if force else "order-free")
        outs.append({"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()})
    assert_same(outs[0], outs[1], f"free-vs-ordered {mode} g={gouraud}")


def _bands(H, n, r, th=32, slots=None):
    """Rows owned by shard r of n (tile row ty -> pattern[ty % period])."""
    from libnativecpurenderer_amd import sharding
    pat = sharding.band_pattern(n, slots)
    return [y for y in range(H) if pat[(y // th) % len(pat)] == r]


def _set_shard(ctx, n, r, slots):
    if slots is None:
        ctx.set_shard(n, r)
    else:
        ctx.set_shard_slots(n, r, slots)


@pytest.mark.parametrize("nshards,slots", [(2, None), (3, None), (8, None), (2, [3, 1]), (3, [1, 4, 2]),
                                           (8, [5, 2, 2, 2, 2, 2, 2, 2])])
@pytest.mark.parametrize("opaque", [True, False])
def test_sharded_frames_assemble_to_the_full_frame(gpu, nshards, slots, opaque):
    """Every shard renders only its tile rows (equal shards, or weighted
    SetShardSlots patterns); the owned rows of all shards put together are
    byte-identical to the unsharded frame (colour + depth), for both
    rasterisers; fragment counts add up; the library's band pattern is the
    host helper's."""
    W, H = 333, 250
    alpha = None if opaque else (0.3, 0.9)
    xy, z, c = scenes.triangle_soup(3000, W, H, 18, seed=41, gouraud=True, alpha=alpha)

    def render(n, r):
        ctx = gpu.context(W, H, False)
        _set_shard(ctx, n, r, slots if n > 1 else None)
        if n > 1:
            from libnativecpurenderer_amd import sharding
            assert ctx.get_shard_pattern() == sharding.band_pattern(n, slots)
        ctx.set_color(0.1, 0.1, 0.1, 0.1)
        ctx.set_depth_state(True, True)
        ctx.clear_depth()
        ctx.set_fragment_counting(True)
        ctx.draw_triangles(xy, c, z=z)
        ctx.gather_frame_u8()           # local conversion of the owned rows
        return ctx.get_buffer_numpy(), ctx.get_depth_buffer(), ctx.get_frame_u8(), ctx.get_fragment_count()

    full, fullz, fullu8, fullfrags = render(1, 0)
    asm, asmz, asmu8 = np.zeros_like(full), np.zeros_like(fullz), np.zeros_like(fullu8)
    frags = 0
    for r in range(nshards):
        f, zz, u8, fr = render(nshards, r)
        rows = _bands(H, nshards, r, slots=slots)
        asm[rows], asmz[rows], asmu8[rows] = f[rows], zz[rows], u8[rows]
        frags += fr
    assert scenes.bits_equal(asm, full)
    assert np.array_equal(asmz, fullz)
    assert np.array_equal(asmu8, fullu8)
    assert frags == fullfrags
    ctx = gpu.context(W, H, False)
    ctx.set_color(0.1, 0.1, 0.1, 0.1)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    ctx.draw_triangles(xy, c, z=z)
    assert np.array_equal(fullu8, ctx.get_buffer_as_uint8_numpy())


@pytest.mark.parametrize("nshards,root,W,H,alpha,slots", [(2, 0, 333, 250, False, None), (3, 1, 333, 250, True, None),
                                                           (8, 0, 256, 300, False, None), (8, 5, 100, 40, False, None),
                                                           (2, 0, 256, 500, False, [5, 1]),
                                                           (4, 2, 333, 700, True, [1, 2, 6, 3]),
                                                           (8, 0, 512, 1000, False, [6, 2, 2, 2, 2, 2, 2, 2]),
                                                           (3, 1, 334, 250, False, None)])
@pytest.mark.parametrize("fmt", ["rgb", "yuv420p"])
@pytest.mark.parametrize("via", ["copy", "rccl"])
def test_packed_band_gather_assembles_the_frame(gpu, nshards, root, W, H, alpha, slots, fmt, via):
    """GatherFrameU8's assembly (each rank's bands packed into one message,
    one unpack on the root), run for n shards on one GPU with device copies
    (via="copy") or RCCL send/recv pairs over a one-rank communicator (via=
    "rccl": GatherFrameU8's group calls on the hardware) in place of the
    inter-process transfers: the root's frame output (u8 image, or its YUV420P
    planes: a band's Y rows and its U and V rows) equals the unsharded frame
    byte for byte (odd widths take the byte-wise copy, multiples of 16 the
    vector one)."""
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    if fmt == "yuv420p" and (W % 2 or H % 2):
        pytest.skip("YUV420P needs even sizes")
    if via == "rccl":
        comm = R.Comm(1, 0, R.Comm.unique_id())

        def gather(ctxs, root):
            R.RenderContext.gather_frame_u8_local_rccl(ctxs, comm, root)
    else:
        gather = R.RenderContext.gather_frame_u8_local
    xy, z, c = scenes.triangle_soup(2000, W, H, 18, seed=43, gouraud=True)

    def render(n, r):
        ctx = gpu.context(W, H, alpha)
        ctx.set_frame_format(fmt)
        _set_shard(ctx, n, r, slots if n > 1 else None)
        ctx.set_color(0.2, 0.1, 0.3, 1.0)
        ctx.set_depth_state(True, True)
        ctx.clear_depth()
        ctx.draw_triangles(xy, c, z=z)
        return ctx

    ref = render(1, 0)
    ref.gather_frame_u8()
    want = ref.get_frame_u8()
    if fmt == "yuv420p":   # the raster's fused planes = the restatement of its u8 image
        assert np.array_equal(want, scenes.yuv420p(ref.get_buffer_as_uint8_numpy()))
    ctxs = [render(nshards, r) for r in range(nshards)]
    gather(ctxs, root)
    got = ctxs[root].get_frame_u8()
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    # more frames: the assembly alternates between two frame buffers and
    # overlaps the next frame (gather stream), so frames 3+ reuse buffers
    # whose earlier transfer must have finished
    for f in range(4):
        for ctx in (ref, *ctxs):
            if f % 2:
                ctx.fill_color(0.5, 0.25 * f, 0.75, 0.5)
            else:
                ctx.set_color(0.1 * f, 0.2, 0.3, 1.0)
                ctx.clear_depth()
                ctx.draw_triangles(xy[f * 300:], c[f * 300:], z=z[f * 300:])
        ref.gather_frame_u8()
        gather(ctxs, root)
        got = ctxs[root].get_frame_u8()
        want = ref.get_frame_u8()
        assert np.array_equal(got, want), (f, np.argwhere(got != want)[:5])


def test_single_rank_comm_gather(gpu):
    """The RCCL path with a one-rank communicator (a no-op assembly)."""
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    comm = R.Comm(1, 0, R.Comm.unique_id())
    ctx = gpu.context(100, 70, True)
    ctx.set_color(0, 0, 0, 0)
    ctx.draw_rect(10, 10, 50, 30, 0.5, 0.25, 1.0, 1.0)
    ctx.gather_frame_u8(comm, 0)
    ctx.gather_framebuffer(comm, 0)
    assert np.array_equal(ctx.get_frame_u8(), ctx.get_buffer_as_uint8_numpy())


@pytest.mark.parametrize("fmt", ["rgb", "yuv420p"])
@pytest.mark.parametrize("alpha", [False, True])
def test_fused_frame_output_matches_conversion(gpu, fmt, alpha):
    """After the first GatherFrameU8 the resolve writes the frame output
    itself (u8 image, or its YUV420P planes); it must equal GetBufferAsUInt8
    (resp. the YUV420P restatement of it) every frame, including frames with a
    second (non-clearing) batch, a primitive drawn after the triangles, a
    blended batch after an opaque one (ordered raster: converted after it), or
    a blended batch right after the clear (the ordered raster's write-back
    produces the frame output itself)."""
    W, H = 300, 200
    xy, z, c = scenes.triangle_soup(2000, W, H, 15, seed=51, gouraud=True)
    bxy, bz, bc = scenes.triangle_soup(600, W, H, 40, seed=52, gouraud=False, alpha=(0.2, 0.8))
    ctx = gpu.context(W, H, alpha)
    ctx.set_frame_format(fmt)
    conv = (lambda a: a) if fmt == "rgb" else scenes.yuv420p
    for frame in range(7):
        ctx.set_color(0.05 * frame, 0.05 * frame, 0.05 * frame, 0.05 * frame)
        ctx.set_depth_state(True, True)
        ctx.clear_depth()
        if frame >= 5:   # ordered raster with the pending clear (Z test off / on without write)
            ctx.set_depth_state(frame == 6, False)
            ctx.draw_triangles(bxy, bc, z=bz, gouraud=False)
            ctx.gather_frame_u8()
            assert np.array_equal(ctx.get_frame_u8(), conv(ctx.get_buffer_as_uint8_numpy())), frame
            continue
        ctx.draw_triangles(xy, c, z=z)
        if frame == 2:
            ctx.draw_triangles(xy[:100] + 7.0, c[:100], z=z[:100] * 0.5)
        if frame == 3:
            ctx.draw_rect(20, 20, 50, 40, 1, 0, 0, 0.5)
        if frame == 4:
            cb = c.copy()
            cb[:, 3::4] = 0.5
            ctx.draw_triangles(xy[:300], cb[:300], z=z[:300])
        ctx.gather_frame_u8()
        assert np.array_equal(ctx.get_frame_u8(), conv(ctx.get_buffer_as_uint8_numpy())), frame


def test_pair_list_overflow_is_rerun_in_order(gpu, oracle):
    """The visibility raster sizes its pair list from an estimate and checks it
    on the device; an overflowing batch does nothing and is re-run, before any
    later call, with an exact allocation.  Force that with a tiny capacity and
    interleave other operations: the frame must still equal the oracle's."""
    W, H = 260, 190
    xy, z, c = scenes.triangle_soup(1500, W, H, 25, seed=61, gouraud=True)
    outs = []
    for fac in (gpu, oracle):
        ctx = fac.context(W, H, True)
        if fac is gpu:
            ctx.set_pair_capacity_override(50)
        ctx.set_color(0.2, 0.2, 0.2, 0.2)
        ctx.set_depth_state(True, True)
        ctx.clear_depth()
        ctx.draw_triangles(xy, c, z=z)                   # overflows -> re-run at the next call
        ctx.draw_rect(30, 30, 80, 60, 0.9, 0.1, 0.1, 0.5)
        ctx.set_color(0.4, 0.4, 0.4, 0.4)                # pending clear after an overflowed batch
        ctx.draw_triangles(xy[::-1], c[::-1], z=z[::-1])
        ctx.draw_triangles(xy[:200] + 3.5, c[:200], z=z[:200])
        outs.append({"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()})
    assert_same(outs[0], outs[1], "overflow")


def test_device_batch_overflow_never_rereads_caller_arrays(gpu, oracle):
    """DrawTrianglesDevice on the caller's HBM tensors with an overflowing pair
    list: the batch is sized exactly inside the call, so once the caller has
    synchronised it may rewrite (or free) the tensors -- the next call on the
    context must not re-run the batch from them."""
    import torch
    W, H = 260, 190
    xy, z, c = scenes.triangle_soup(1500, W, H, 25, seed=62, gouraud=True)
    want = {}
    octx = oracle.context(W, H, False)
    octx.set_color(0.2, 0.2, 0.2, 0.2)
    octx.set_depth_state(True, True)
    octx.clear_depth()
    octx.draw_triangles(xy, c, z=z)
    octx.draw_rect(30, 30, 80, 60, 0.9, 0.1, 0.1, 0.5)
    want = {"f64": octx.get_buffer_numpy(), "depth": octx.get_depth_buffer()}
    dxy, dz, dc = (torch.from_numpy(np.ascontiguousarray(a, np.float64).ravel()).to("cuda") for a in (xy, z, c))
    torch.cuda.synchronize()
    ctx = gpu.context(W, H, False)
    ctx.set_pair_capacity_override(50)
    ctx.set_color(0.2, 0.2, 0.2, 0.2)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    ctx.draw_triangles_device(dxy, dc, len(xy), z=dz, gouraud=True)
    torch.cuda.synchronize()
    dxy.fill_(float("nan")); dz.zero_(); dc.zero_()      # the caller reuses its tensors
    torch.cuda.synchronize()
    ctx.draw_rect(30, 30, 80, 60, 0.9, 0.1, 0.1, 0.5)
    assert_same({"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()}, want, "device overflow")


def test_rotate_uses_sincos_like_the_reference_build(gpu, oracle):
    """cpp:436-444 compiled by g++ -O3 (src/compile.sh) calls glibc sincos(),
    which differs from separate sin/cos in the last bit for some angles: the
    transform state after many rotations must equal the oracle's (gcc) bit
    for bit."""
    import numpy as np
    r = np.random.Generator(np.random.PCG64(99))
    g, o = gpu.context(8, 8, False), oracle.context(8, 8, False)
    for a in r.uniform(-0.5, 0.5, 2000):
        g.set_transform(1, 0, 0, 1, 0, 0)
        o.set_transform(1, 0, 0, 1, 0, 0)
        g.rotate(float(a))
        o.rotate(float(a))
        assert g.get_transform() == o.get_transform(), a


@pytest.mark.parametrize("shape", [(128, 128), (96, 40)])
def test_hit_effect_textures_match_oracle(gpu, shape):
    """Helpers.create_milthm_hit_effect_textures (Pybind:34-48, cpp:1318-1440):
    n textures of one mask/seed from one launch equal the oracle's textures
    texel for texel (binary alpha x mask alpha, column-major storage).  The
    device sin/atan2 are within an ULP of glibc's; that can only flip a texel
    whose noise lies within ~1e-11 of the threshold, which none of these do."""
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    w, h = shape
    if shape == (128, 128):
        mask = np.load(os.path.join(scenes.ROOT, "tests", "golden", "image_png_rgba.npy"))
    else:
        mask = scenes.hit_mask(w, h, seed=11)
    n, seed = 6, 0.6180339887
    texs = R.Helpers.create_milthm_hit_effect_textures(R.Texture.from_numpy(mask), n, seed=seed)
    assert len(texs) == n
    for i, tex in enumerate(texs):
        assert (tex.width, tex.height, tex.enableAlpha) == (w, h, True)
        got = tex.get_buffer_numpy().reshape(h, w, 4)
        want = scenes.oracle_hit_effect(mask, seed, i / (n - 1))
        assert scenes.bits_equal(got, want), scenes.first_mismatch(got, want)
    # the single-texture entry point (h:151) and the inline pixel function (h:150)
    mtex = R.Texture.from_numpy(mask)
    single = R.PtrCreatedTexture(R.lib.CreateMilthmHitEffectTexture(mtex._ptr, seed, 0.3, 0.1, 0.2, 0.3))
    want = scenes.oracle_hit_effect(mask, seed, 0.3, rgb=(0.1, 0.2, 0.3))
    assert scenes.bits_equal(single.get_buffer_numpy().reshape(h, w, 4), want)
    a = ctypes.c_double()
    for x, y in [(0.1, 0.2), (0.75, 0.6), (0.5, 0.5)]:
        R.lib.GetMilthmHitEffectPixel(seed, 0.4, x, y, ctypes.byref(a))
        b = ctypes.c_double()
        scenes._OracleLib.get().GetMilthmHitEffectPixel(seed, 0.4, x, y, ctypes.byref(b))
        assert a.value == b.value


def test_hit_effect_needs_alpha_mask(gpu):
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    tex = R.Texture.from_numpy(np.zeros((8, 8, 3), dtype=np.uint8))
    assert not R.lib.CreateMilthmHitEffectTexture(tex._ptr, 0.1, 0.5, 1.0, 1.0, 1.0)


@pytest.mark.parametrize("deliver", ["none", "bands"])
def test_bench_multi_rank_orchestration_on_one_gpu(gpu, tmp_path, deliver):
    """bench.py's N>1 path (torchrun, 2 ranks): partition calibration over
    weighted shards, barriers, max-over-ranks timing and the JSON line -- run
    with a gloo group and every rank on this one GPU (--gloo-test skips only the
    RCCL frame gather, which needs one GPU per rank).  deliver=bands: each rank
    copies its bands into two shared pinned host frames (DeliverFrameBands)."""
    import json
    import socket
    import subprocess
    import sys
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(scenes.ROOT, "bench.py"),
           "--gpus", "2", "--steps", "5", "--warmup", "1", "--gloo-test", "--config", "c2", "--deliver", deliver]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    assert out.returncode == 0, out.stderr[-3000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["steps"] == 5
    assert set(d["config"]["partition_calibration_ms"]) >= {"equal", "3", "12"}
    # the last timed frame of every rank checked against the oracle's digests
    assert d["verified"] is True and d["warm_failures"] == 0, {k: d.get(k) for k in ("verify_mismatches", "verify_note")}
    if deliver == "bands":
        assert "shared pinned host frame" in d["config"]["frame_delivery"]


@pytest.mark.parametrize("alpha", [False, True])
def test_frame_yuv420p_matches_restatement(gpu, alpha):
    """GetFrameYUV420P (§8f-2) converts the gathered u8 frame on the GPU:
    equal, byte for byte, to the numpy restatement applied to the same frame
    (and to the oracle's u8 image of the same scene)."""
    W, H = 322, 190
    xy, z, c = scenes.triangle_soup(1500, W, H, 25, seed=5, gouraud=True)
    outs = {}
    for fac in (gpu, scenes.OracleFactory()):
        ctx = fac.context(W, H, alpha)
        ctx.set_color(0.1, 0.6, 0.3, 1.0)
        ctx.set_depth_state(True, True)
        ctx.clear_depth()
        ctx.draw_triangles(xy, c, z=z)
        ctx.draw_rect(10, 10, 100, 60, 1.0, 0.2, 0.1, 0.5)
        outs[fac.name] = ctx
    g = outs["gpu"]
    g.gather_frame_u8()
    got = g.get_frame_yuv420p()
    want = scenes.yuv420p(outs["oracle"].get_buffer_as_uint8_numpy())
    assert np.array_equal(got, want), np.argwhere(got != want)[:5]
    assert np.array_equal(scenes.yuv420p(g.get_frame_u8()), want)
    odd = gpu.context(5, 4, False)
    odd.gather_frame_u8()
    with pytest.raises(RuntimeError):
        odd.get_frame_yuv420p()


def test_resize_drops_the_gathered_frame(gpu):
    """ResizeRenderContext drops the gathered frame (its buffers hold the old
    size): get_frame_u8 raises until the next gather instead of returning an
    unwritten buffer; an odd size resets YUV420P to the u8 image visibly (an
    error message is latched) and the next gather is the u8 image."""
    from libnativecpurenderer_amd import _lib
    ctx = gpu.context(64, 48, False)
    with pytest.raises(RuntimeError):
        ctx.get_frame_u8()                     # nothing gathered yet
    ctx.set_frame_format("yuv420p")
    ctx.set_color(0.5, 0.25, 0.75, 1.0)
    ctx.gather_frame_u8()
    assert ctx.get_frame_u8().size == 64 * 48 * 3 // 2
    ctx.resize(96, 64)
    with pytest.raises(RuntimeError):
        ctx.get_frame_u8()
    _lib.clear_error()
    ctx.resize(33, 20)
    assert "YUV420P" in _lib.last_error()
    ctx.set_color(0.5, 0.25, 0.75, 1.0)
    ctx.gather_frame_u8()
    assert np.array_equal(ctx.get_frame_u8(), ctx.get_buffer_as_uint8_numpy())


@pytest.mark.parametrize("fmt", ["rgb", "yuv420p"])
def test_delivered_frames_match_the_frames(gpu, fmt):
    """DeliverFrameU8 (frame k's D2H on the gather stream into pinned host
    buffers, overlapped with frame k+1's render; two host buffers in
    rotation): every delivered frame equals that frame's output read back
    synchronously from a second context rendering the same sequence."""
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    W, H = 320, 192
    xy, z, c = scenes.triangle_soup(4000, W, H, 20, seed=77, gouraud=True)
    buf = R.TriangleBuffer(xy, c, z=z, gouraud=True)
    ctx, ref = gpu.context(W, H, False), gpu.context(W, H, False)
    for cx in (ctx, ref):
        cx.set_frame_format(fmt)
        cx.set_depth_state(True, True)
    shape = ctx.frame_output_shape()
    host = [R.HostBuffer(int(np.prod(shape))) for _ in range(2)]
    pending, got, want = None, [], []

    def draw(cx, f):
        cx.set_color(0.1 * f, 0.05, 0.2, 1.0)
        cx.clear_depth()
        cx.set_transform(1, 0, 0, 1, 3.0 * f, -2.0 * f)
        cx.draw_triangle_buffer(buf)
        cx.gather_frame_u8()

    for f in range(7):
        draw(ctx, f)
        t = ctx.deliver_frame(host[f % 2])
        draw(ref, f)
        want.append(ref.get_frame_u8().copy())
        if pending is not None:
            ctx.wait_frame_delivered(pending[0])
            got.append(host[pending[1]].array(shape).copy())
        pending = (t, f % 2)
    ctx.wait_frame_delivered(pending[0])
    got.append(host[pending[1]].array(shape).copy())
    for f in range(7):
        assert np.array_equal(got[f], want[f]), (f, np.argwhere(got[f] != want[f])[:5])
    assert not np.array_equal(want[0], want[1])


@pytest.mark.parametrize("limits", [(64, 64), (200, 96), (512, 256)])
def test_split_dense_tiles_match_oracle(gpu, oracle, limits):
    """Dense tiles split into slices (SetSplitLimits: tiles of more than
    split_at pairs cut into slices of ~dslice pairs), each slice's keys in its
    own slot, the last slice reducing them and shading: every depth mode, RGB
    and RGBA, flat and Gouraud, against the oracle -- from ~1000 pairs per tile
    (up to 16 slices a tile) down to tiles just over the limit."""
    W, H = 256, 160
    dense = scenes.triangle_soup(20000, W, H, 3, seed=91, gouraud=True)
    big = scenes.triangle_soup(200, W, H, 60, seed=92, gouraud=True)
    xy = np.concatenate([dense[0], big[0]]); z = np.concatenate([dense[1], big[1]])
    c = np.concatenate([dense[2], big[2]])
    perm = np.random.Generator(np.random.PCG64(93)).permutation(len(xy))
    xy, z, c = xy[perm], z[perm], c[perm]
    for depth, write in ((True, True), (True, False), (False, True)):
        for alpha in (False, True):
            for gouraud in (True, False):
                cc = c if gouraud else c[:, :4]
                outs = []
                for fac in (gpu, oracle):
                    ctx = fac.context(W, H, alpha)
                    if fac is gpu:
                        ctx.set_split_limits(*limits)
                    ctx.set_color(0.25, 0.25, 0.25, 0.25)
                    ctx.set_depth_state(depth, write)
                    ctx.clear_depth()
                    ctx.draw_triangles(xy, cc, z=z)
                    ctx.draw_triangles(xy[::3] + 0.5, cc[::3], z=z[::3] * 0.5)   # a second batch over the first
                    outs.append({"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()})
                assert_same(outs[0], outs[1], f"split {limits} depth={depth} write={write} alpha={alpha} g={gouraud}")


def _warm_frames(fac, W, H, parts, warm):
    """A TriangleBuffer (GPU; the same arrays on the oracle) drawn frame after
    frame: repeats under one binning key bin warm (one pass into the kept tile
    ranges), a transform change or a different buffer bins cold again and
    re-captures, a return to the first key is warm again.  The mesh has dense
    tiles (split work items) and empty ones."""
    mesh, blob = parts
    ctx = fac.context(W, H, False)
    if warm is not None:
        ctx.set_warm_binning(warm)
    bufs = None
    if fac.name == "gpu":
        from libnativecpurenderer_amd import libNativeCPURendererPybind as R
        bufs = [R.TriangleBuffer(p[0], p[2], z=p[1], gouraud=True) for p in parts]
    outs = []
    for which, xf in [(0, 0), (0, 0), (0, 0), (0, 1), (0, 1), (0, 0), (1, 0), (1, 0), (0, 0), (0, 0)]:
        ctx.save_state()
        if xf:
            ctx.translate(3.5, -2.25)
            ctx.scale(1.1, 0.9)
        ctx.set_color(0.1, 0.1, 0.1, 0.1)
        ctx.set_depth_state(True, True)
        ctx.clear_depth()
        if bufs is not None:
            ctx.draw_triangle_buffer(bufs[which])
        else:
            p = parts[which]
            ctx.draw_triangles(p[0], p[2], z=p[1])
        ctx.restore_state()
        outs.append({"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()})
    return outs, (ctx.warm_batch_count() if bufs is not None else None)


def test_warm_binning_frames(gpu, oracle):
    W, H = 640, 400
    mesh = scenes.sphere_mesh(W, H, 100, 300)
    xy, z, c = scenes.triangle_soup(4000, 60, 40, 3.0, seed=77, gouraud=True)   # one dense tile: split items
    blob = (xy + np.array([200.0, 100.0] * 3), z, c)
    both = (np.concatenate([mesh[0], blob[0]]), np.concatenate([mesh[1], blob[1]]), np.concatenate([mesh[2], blob[2]]))
    parts = (both, mesh)
    want, _ = _warm_frames(oracle, W, H, parts, None)
    got, nwarm = _warm_frames(gpu, W, H, parts, 1)
    for k, (g, o) in enumerate(zip(got, want)):
        assert_same(g, o, f"warm frame {k}")
    assert nwarm >= 4, nwarm   # frames 2, 4, 7 and 9 at least (each after a validated draw under its key)
    cold, ncold = _warm_frames(gpu, W, H, parts, 2)
    assert ncold == 0
    for k, (g, o) in enumerate(zip(cold, want)):
        assert_same(g, o, f"cold frame {k}")
