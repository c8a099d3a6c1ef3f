"""Deferred command list (include/libNativeCPURenderer.h
BeginCommandList): every scene's primitive draws recorded and run as one
launch must give the oracle's sequential result bit for bit, and the list
must run before anything that reads or overwrites the framebuffer."""
import numpy as np
import pytest

import scenes
from test_parity_gpu import assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def recording():
    return scenes.GpuRecordingFactory()


@pytest.mark.parametrize("name", sorted(n for n in scenes.all_scenes() if not n.startswith("tri_")))
def test_recorded_scene_parity(recording, oracle, golden, name):
    g = scenes.run_scene(name, recording)
    o = scenes.run_scene(name, oracle)
    assert_same(g, o, f"recorded {name}")
    for k, v in g.items():
        assert scenes.bits_equal(v, golden[f"{name}/{k}"]), f"recorded {name}/{k} vs golden"


@pytest.mark.parametrize("alpha", [False, True])
@pytest.mark.parametrize("seed", [31, 32, 33])
def test_recorded_mix_large(recording, oracle, alpha, seed):
    """Larger frames than the tile (64x16) with many commands, ragged size."""
    kw = dict(W=333, H=157, alpha=alpha, n=600, seed=seed, flushes=seed == 33)
    assert_same(scenes.scene_primitive_mix(recording, **kw), scenes.scene_primitive_mix(oracle, **kw),
                f"mix seed={seed} alpha={alpha}")


def test_list_lifecycle(gpu):
    ctx = gpu.context(70, 40, False)
    ctx.set_color(0.2, 0.2, 0.2, 0.2)
    assert not ctx.is_recording()
    ctx.begin_commands()
    assert ctx.is_recording()
    ctx.draw_rect(3, 4, 20, 10, 1, 0, 0, 1)
    ctx.draw_circle(30, 20, 8, 0, 1, 0, 0.5)
    ctx.fill_color(0, 0, 1, 0.25)
    assert ctx.command_list_length() == 3
    c = ctx.get_color(5, 5)            # a readback runs the queue first
    assert ctx.command_list_length() == 0 and ctx.is_recording()
    assert c[0] > 0.5
    ctx.draw_rect(0, 0, 70, 40, 1, 1, 1, 1)
    ctx.set_color(0.5, 0.5, 0.5, 0.5)  # overwrites everything: the queue is dropped
    assert ctx.command_list_length() == 0
    ctx.draw_line(0, 0, 69, 39, 3, 1, 0, 1, 1)
    ctx.flush_commands()
    assert ctx.command_list_length() == 0 and ctx.is_recording()
    ctx.end_commands()
    assert not ctx.is_recording()
    ref = gpu.context(70, 40, False)
    ref.set_color(0.5, 0.5, 0.5, 0.5)
    ref.draw_line(0, 0, 69, 39, 3, 1, 0, 1, 1)
    assert scenes.bits_equal(ctx.get_buffer_numpy(), ref.get_buffer_numpy())


def test_texture_destroyed_while_queued(gpu, oracle):
    """A queued draw keeps sampling a texture the caller releases before the
    list runs (DestroyTexture runs every queue first)."""
    outs = []
    for fac in (gpu, oracle):
        ctx = fac.context(50, 30, True)
        if fac is gpu:
            ctx.begin_commands()
        ctx.set_color(0, 0, 0, 0)
        tex = fac.texture(scenes.pattern_u8(12, 10, 4, seed=5))
        ctx.draw_texture(tex, 4, 3, 40, 22)
        del tex
        outs.append(ctx.get_buffer_numpy())
    assert scenes.bits_equal(outs[0], outs[1]), scenes.first_mismatch(outs[0], outs[1])


def test_recording_context_frames(gpu, oracle):
    """RecordingRenderContext (the reference proxy's counterpart): a frame's
    draws replay at end_of_frame()."""
    R = gpu.R
    ctx = R.RecordingRenderContext(64, 48, False)
    ref = oracle.context(64, 48, False)
    for f in range(3):
        for c in (ctx, ref):
            c.set_color(0, 0, 0, 0)
            c.draw_rect(5 + f, 6, 30, 20, 0.3 * f, 0.5, 0.9, 0.7)
            c.draw_vertical_grd(0, 0, 64, 48, 1, 0, 0, 0.3, 0, 0, 1, 0.6)
        assert ctx.command_list_length() == 2
        ctx.end_of_frame()
        assert ctx.command_list_length() == 0
        assert scenes.bits_equal(ctx.get_buffer_numpy(), ref.get_buffer_numpy()), f
    assert ctx.frames == 3


@pytest.mark.parametrize("recording", [False, True])
@pytest.mark.parametrize("name", sorted(n for n in scenes.all_scenes() if not n.startswith("tri_")))
def test_packed_scene_parity(oracle, golden, name, recording):
    """Every primitive scene through PackedCommands (one ExecuteCommands array
    per run of draw / state calls), immediate and inside a command list."""
    g = scenes.run_scene(name, scenes.GpuPackedFactory(recording))
    o = scenes.run_scene(name, oracle)
    assert_same(g, o, f"packed {name}")


@pytest.mark.parametrize("alpha", [False, True])
@pytest.mark.parametrize("seed", [41, 42])
def test_packed_mix_large(oracle, alpha, seed):
    kw = dict(W=333, H=157, alpha=alpha, n=600, seed=seed, flushes=seed == 42)
    assert_same(scenes.scene_primitive_mix(scenes.GpuPackedFactory(True), **kw),
                scenes.scene_primitive_mix(oracle, **kw), f"packed mix seed={seed} alpha={alpha}")


def test_execute_commands_rejects_malformed_arrays(gpu):
    """A malformed array runs its commands up to the bad one and reports -1
    with a latched error: unknown opcode, truncated command, texture index out
    of range, fractional pixel coordinate."""
    import ctypes
    from libnativecpurenderer_amd import _lib
    lib = _lib.load()
    tex = gpu.texture(scenes.pattern_u8(8, 8, 4, seed=3))
    texs = (ctypes.c_void_p * 1)(tex._ptr)

    def run(words):
        ctx = gpu.context(32, 16, False)
        ctx.set_color(0, 0, 0, 0)
        arr = np.asarray(words, dtype=np.float64)
        _lib.clear_error()
        n = lib.ExecuteCommands(ctx._ptr, arr.ctypes.data, len(arr), texs, 1)
        return n, _lib.last_error(), ctx.get_buffer_numpy()

    rect = [13, 0, 0, 8, 8, 1, 0, 0, 1]           # DrawRect: red 8x8
    n, err, fb = run(rect + [99])
    assert n == -1 and "unknown opcode" in err and fb[2, 2, 0] == 1.0
    n, err, fb = run(rect + [13, 0, 0, 4])
    assert n == -1 and "truncated" in err and fb[2, 2, 0] == 1.0
    n, err, fb = run(rect + [11, 1, 0, 0, 8, 8])
    assert n == -1 and "texture index" in err
    n, err, fb = run(rect + [17, 1.5, 2, 0, 1, 0, 1])
    assert n == -1 and "pixel coordinate" in err
    n, err, fb = run(rect + [11, 0, 10, 0, 8, 8] + [5, 1.0, 2.0])   # + a texture and a translate: 3 commands
    assert n == 3 and err == ""
