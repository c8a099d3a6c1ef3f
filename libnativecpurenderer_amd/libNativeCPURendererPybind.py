"""Drop-in mirror of the reference's ctypes module
(/root/reference/src/libNativeCPURendererPybind.py) for the raster path,
backed by the HIP library libNativeCPURenderer.so built for gfx950.

Same class names, method names, arities and argument meaning as the
reference (RenderContext :51-300, Texture :369-435, PtrCreatedTexture
:437-440, Helpers :11-49, get_version :661-666), so
``import libnativecpurenderer_amd.libNativeCPURendererPybind as CPURenderer``
replaces ``import libNativeCPURendererPybind as CPURenderer``
(milrenderer.py:17) for every raster call.  Additions (triangles, depth,
numpy readback, timing) are new methods; nothing existing changes meaning.

Deliberate differences from the reference binding, each a reference bug:
  * get_color passes f64 coordinates (the reference declares c_long for the
    f64 parameters of GetColor, h:113, and crashes — SURVEY §8b);
  * Texture(..., is_uint8=False) works (the reference's
    `c_double * len(data) // 8` precedence bug raises TypeError, :391);
  * apply_pixel works (the reference .so does not export ApplyPixel);
  * AudioClip.overlay(..., time_unit="frame") passes the frame as an integer
    (the reference declares c_double for OverlayAudioClip's i64, Pybind:580,
    so the bool lands in the frame register) and AudioClip(rate, ch, data)
    counts frames as len(data) // channels (the reference passes len(data),
    Pybind:510, and reads past the buffer for ch > 1).
Out of scope here (media back-end): VideoCap (FFmpeg).
"""
from __future__ import annotations

import ctypes
import random
import math
import typing

import numpy as np

from . import _lib

lib = _lib.load()


def _check(ptr, what: str):
    if not ptr:
        raise RuntimeError(f"{what} failed: {_lib.last_error() or 'no HIP device / allocation failure'}")
    return ptr


def _f64_ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class Helpers:
    @staticmethod
    def get_wappered_bytes_data_ptr(bytes: int):
        return lib.GetWapperedBytesDataPtr(bytes)

    @staticmethod
    def get_wappered_bytes_data_size(bytes: int):
        return lib.GetWapperedBytesDataSize(bytes)

    @staticmethod
    def wappered_bytes_to_python(bytes: int):
        """Pybind:29-32; the WapperedBytes are released after the copy (the
        reference leaks them)."""
        ptr = Helpers.get_wappered_bytes_data_ptr(bytes)
        size = Helpers.get_wappered_bytes_data_size(bytes)
        out = ctypes.string_at(ptr, size)
        lib.DestroyWapperedBytes(bytes)
        return out

    @staticmethod
    def create_milthm_hit_effect_textures(mask: "Texture", n: int, seed: typing.Optional[float] = None):
        """n hit-effect textures of `mask` at thresholds i / (n - 1) with one
        random seed and the colour #9690fd (Pybind:34-48), made by one launch
        (CreateMilthmHitEffectTextures).  `seed` (new, keyword) fixes the seed;
        n == 1 raises ZeroDivisionError like the reference."""
        if seed is None:
            seed = random.random()
        ts = [i / (n - 1) for i in range(n)]
        arr = (ctypes.c_double * max(n, 1))(*ts)
        out = (ctypes.c_void_p * max(n, 1))()
        if not lib.CreateMilthmHitEffectTextures(mask._ptr, seed, arr, n, 0x96 / 0xff, 0x90 / 0xff, 0xfd / 0xff, out):
            raise RuntimeError("CreateMilthmHitEffectTextures failed (mask without alpha?) " + _lib.last_error())
        return [PtrCreatedTexture(out[i]) for i in range(n)]


class RenderContext:
    """Framebuffer in HBM + host-side transform/colour state (cpp:3-45)."""

    def __init__(self, width: int, height: int, enable_alpha: bool):
        self.width = width
        self.height = height
        self.enable_alpha = enable_alpha
        self._can_release = False
        self._ptr = _check(lib.CreateRenderContext(width, height, enable_alpha), "CreateRenderContext")
        self._can_release = True

    def __del__(self):
        if not getattr(self, "_can_release", False):
            return
        lib.DestroyRenderContext(self._ptr)
        self._ptr = 0
        self._can_release = False

    # ---- readback -------------------------------------------------------
    def get_buffer_size(self):
        return lib.GetBufferSize(self._ptr)

    def get_buffer(self):
        return self.get_buffer_numpy().tolist()

    def get_buffer_as_uint8(self):
        buffer = bytearray(self.get_buffer_size())
        lib.GetBufferAsUInt8(self._ptr, (ctypes.c_byte * len(buffer)).from_buffer(buffer))
        return buffer

    # ---- pixel ops -----------------------------------------------------
    def fill_color(self, r: float, g: float, b: float, a: float):
        lib.FillColor(self._ptr, r, g, b, a)

    def draw_texture(self, tex: "Texture", x: float, y: float, w: float, h: float):
        lib.DrawTexture(self._ptr, tex._ptr, x, y, w, h)

    def resize(self, width: int, height: int):
        lib.ResizeRenderContext(self._ptr, width, height)
        self.width = width
        self.height = height

    def draw_splitted_texture(self, tex: "Texture", x: float, y: float, width: float, height: float,
                              u_start: float, u_end: float, v_start: float, v_end: float):
        lib.DrawSplittedTexture(self._ptr, tex._ptr, x, y, width, height, u_start, u_end, v_start, v_end)

    # ---- transform state -----------------------------------------------
    def apply_transform(self, a: float, b: float, c: float, d: float, e: float, f: float):
        lib.ApplyTransform(self._ptr, a, b, c, d, e, f)

    def scale(self, sx: float, sy: float):
        lib.Scale(self._ptr, sx, sy)

    def rotate(self, angle: float):
        lib.Rotate(self._ptr, angle)

    def translate(self, tx: float, ty: float):
        lib.Translate(self._ptr, tx, ty)

    def rotate_degree(self, deg: float):
        self.rotate(deg * math.pi / 180)

    def save_state(self):
        lib.SaveContextState(self._ptr)

    def restore_state(self):
        lib.RestoreContextState(self._ptr)

    def draw_line(self, x0: float, y0: float, x1: float, y1: float, width: float,
                  r: float, g: float, b: float, a: float):
        lib.DrawLine(self._ptr, x0, y0, x1, y1, width, r, g, b, a)

    def draw_rect(self, x: float, y: float, width: float, height: float, r: float, g: float, b: float, a: float):
        lib.DrawRect(self._ptr, x, y, width, height, r, g, b, a)

    def get_transform(self):
        out = (ctypes.c_double * 6)()
        lib.GetTransform(self._ptr, ctypes.byref(out))
        return tuple(out)

    def get_inverse_transform(self):
        out = (ctypes.c_double * 6)()
        lib.GetInverseTransform(self._ptr, ctypes.byref(out))
        return tuple(out)

    def apply_pixel(self, x: int, y: int, r: float, g: float, b: float, a: float):
        lib.ApplyPixel(self._ptr, x, y, r, g, b, a)

    def draw_circle(self, x: float, y: float, radius: float, r: float, g: float, b: float, a: float):
        lib.DrawCircle(self._ptr, x, y, radius, r, g, b, a)

    def set_transform(self, a: float, b: float, c: float, d: float, e: float, f: float):
        lib.SetTransform(self._ptr, a, b, c, d, e, f)

    def set_color_transform(self, r: float, g: float, b: float, a: float):
        lib.SetColorTransform(self._ptr, r, g, b, a)

    def apply_color_transform(self, r: float, g: float, b: float, a: float):
        lib.ApplyColorTransform(self._ptr, r, g, b, a)

    def set_pixel(self, x: int, y: int, r: float, g: float, b: float, a: float):
        lib.SetPixel(self._ptr, x, y, r, g, b, a)

    def set_color(self, r: float, g: float, b: float, a: float):
        lib.SetColor(self._ptr, r, g, b, a)

    def get_color(self, x: float, y: float):
        out = (ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double())
        lib.GetColor(self._ptr, x, y, *(ctypes.byref(o) for o in out))
        return tuple(o.value for o in out)

    def draw_vertical_grd(self, x: float, y: float, width: float, height: float,
                          top_r: float, top_g: float, top_b: float, top_a: float,
                          bottom_r: float, bottom_g: float, bottom_b: float, bottom_a: float):
        lib.DrawVerticalGrd(self._ptr, x, y, width, height, top_r, top_g, top_b, top_a,
                            bottom_r, bottom_g, bottom_b, bottom_a)

    def draw_vertical_mut_grd(self, x: float, y: float, width: float, height: float,
                              steps: list[tuple[float, tuple[float, float, float, float]]]):
        # Pybind.py:272-280: consecutive stops become DrawVerticalGrd bands
        for i, (p, s) in enumerate(steps):
            if i == len(steps) - 1:
                break
            np_, ns = steps[i + 1]
            ty = y + height * p
            theight = height * (np_ - p)
            self.draw_vertical_grd(x, ty, width, theight, s[0], s[1], s[2], s[3], ns[0], ns[1], ns[2], ns[3])

    def as_texure(self):   # sic: the reference's method name (Pybind.py:282)
        return PtrCreatedTexture(_check(lib.CreateTextureFromRenderContext(self._ptr), "CreateTextureFromRenderContext"))

    def as_texture_shared(self):
        res = PtrCreatedTexture(
            _check(lib.CreateTextureFromRenderContextShared(self._ptr), "CreateTextureFromRenderContextShared"))
        res._can_release = False
        return res

    def as_pilimg(self):
        from PIL import Image
        return Image.frombytes("RGBA" if self.enable_alpha else "RGB", (self.width, self.height),
                               bytes(self.get_buffer_as_uint8()))

    # ---- additions: numpy readback -------------------------------------
    def get_buffer_numpy(self) -> np.ndarray:
        """Framebuffer as a (H, W, ipp) float64 array (one D2H copy)."""
        ipp = 4 if self.enable_alpha else 3
        out = np.empty((self.height, self.width, ipp), dtype=np.float64)
        lib.GetBuffer(self._ptr, _f64_ptr(out))
        return out

    def get_buffer_as_uint8_numpy(self) -> np.ndarray:
        ipp = 4 if self.enable_alpha else 3
        out = np.empty((self.height, self.width, ipp), dtype=np.uint8)
        lib.GetBufferAsUInt8(self._ptr, out.ctypes.data_as(ctypes.c_void_p))
        return out

    # ---- additions: triangles + depth ----------------------------------
    def set_depth_state(self, test: bool, write: bool = True):
        lib.SetDepthState(self._ptr, bool(test), bool(write))

    def clear_depth(self, value: int = 0xFFFFFFFF):
        lib.ClearDepth(self._ptr, value)

    def get_depth_buffer(self) -> np.ndarray:
        out = np.empty((self.height, self.width), dtype=np.uint32)
        lib.GetDepthBuffer(self._ptr, out.ctypes.data_as(ctypes.c_void_p))
        return out

    def draw_triangles(self, xy, rgba, z=None, gouraud: typing.Optional[bool] = None):
        """Draws n triangles in the current transform.

        xy: (n, 3, 2) or (n, 6) vertex positions; rgba: (n, 4) flat colours or
        (n, 3, 4) / (n, 12) per-vertex colours (Gouraud); z: (n, 3) depths in
        [0, 1] or None."""
        xy = np.ascontiguousarray(xy, dtype=np.float64).reshape(-1, 6)
        n = xy.shape[0]
        rgba = np.ascontiguousarray(rgba, dtype=np.float64)
        if gouraud is None:
            gouraud = rgba.size == 12 * n and n > 0
        rgba = rgba.reshape(n, 12 if gouraud else 4)
        if rgba.shape[1] != (12 if gouraud else 4):
            raise ValueError("rgba must hold 4 (flat) or 12 (Gouraud) values per triangle")
        zp = None
        if z is not None:
            z = np.ascontiguousarray(z, dtype=np.float64).reshape(n, 3)
            zp = _f64_ptr(z)
        lib.DrawTriangles(self._ptr, _f64_ptr(xy), zp, _f64_ptr(rgba), n, bool(gouraud))

    def draw_triangles_device(self, xy, rgba, n: int, z=None, gouraud: bool = False):
        """DrawTrianglesDevice: the arrays already live in HBM on this
        context's device.  xy / rgba / z are device addresses (int) or objects
        with .data_ptr() (e.g. torch tensors, contiguous f64); layouts as
        draw_triangles.  The call enqueues work: keep the arrays alive and
        unchanged until the batch has executed (flush, any readback, or a
        device synchronisation such as torch.cuda.synchronize()); nothing
        reads them after that (an overflowing batch is re-sized in the call)."""
        def addr(a):
            if a is None:
                return None
            return a.data_ptr() if hasattr(a, "data_ptr") else int(a)
        lib.DrawTrianglesDevice(self._ptr, addr(xy), addr(z), addr(rgba), int(n), bool(gouraud))

    def draw_triangle_buffer(self, buf: "TriangleBuffer"):
        lib.DrawTriangleBuffer(self._ptr, buf._ptr)

    # ---- additions: sync, device interop, measurement ------------------
    def flush(self):
        lib.Flush(self._ptr)

    @property
    def device(self) -> int:
        return lib.GetContextDevice(self._ptr)

    def device_buffer_ptr(self) -> int:
        """Device address of the f64 framebuffer (GetDeviceBufferPtr: the pending
        clears are written first; the bytes are current once flush() returns)."""
        return lib.GetDeviceBufferPtr(self._ptr)

    def stream_ptr(self) -> int:
        return lib.GetStreamPtr(self._ptr)

    def enable_kernel_timing(self, on: bool = True):
        lib.EnableKernelTiming(self._ptr, on)

    def reset_kernel_timing(self):
        lib.ResetKernelTiming(self._ptr)

    def set_kernel_timing_filter(self, names: str = ""):
        """Time only these kernels (comma-separated names; "" = all)."""
        lib.SetKernelTimingFilter(self._ptr, names.encode())

    def get_kernel_timing(self, name: str):
        """(total_ms, launches) of one kernel since the last reset."""
        tot = ctypes.c_double()
        cnt = ctypes.c_long()
        if not lib.GetKernelTiming(self._ptr, name.encode(), ctypes.byref(tot), ctypes.byref(cnt)):
            raise KeyError(name)
        return tot.value, cnt.value

    def set_fragment_counting(self, on: bool = True):
        lib.SetFragmentCounting(self._ptr, on)

    def get_fragment_count(self) -> int:
        return lib.GetFragmentCount(self._ptr)

    # ---- additions: multi-GPU frames ----------------------
    def set_shard(self, nshards: int, shard: int):
        """Render only the 32-pixel tile rows ty with ty % nshards == shard."""
        lib.SetShard(self._ptr, nshards, shard)

    def set_shard_slots(self, nshards: int, shard: int, slots: typing.Sequence[int]):
        """Weighted shards: rank p owns slots[p] of every sum(slots) (<= 64)
        tile rows, interleaved (SetShardSlots).  Same call on every rank."""
        arr = (ctypes.c_long * nshards)(*[int(v) for v in slots])
        lib.SetShardSlots(self._ptr, nshards, shard, arr)
        err = _lib.last_error()
        if "SetShardSlots" in err:
            raise ValueError(err)

    def get_shard_pattern(self) -> typing.List[int]:
        """Owner rank of tile row ty is pattern[ty % len(pattern)]."""
        buf = (ctypes.c_ubyte * 64)()
        period = lib.GetShardPattern(self._ptr, buf)
        return list(buf[:period])

    def gather_frame_u8(self, comm: typing.Optional["Comm"] = None, root: int = 0):
        """u8 image of the frame assembled on `root` (local conversion when
        comm is None).  Asynchronous; read it with get_frame_u8()."""
        if not lib.GatherFrameU8(self._ptr, comm._ptr if comm is not None else None, root):
            raise RuntimeError("GatherFrameU8 failed: " + _lib.last_error())

    def get_frame_u8(self) -> np.ndarray:
        """The frame output of the last gather: the (H, W, ipp) u8 image, or
        with set_frame_format("yuv420p") the flat Y, U, V planes."""
        if lib.GetFrameFormat(self._ptr) == 1:
            out = np.empty(self.width * self.height + 2 * (self.width // 2) * (self.height // 2), dtype=np.uint8)
        else:
            out = np.empty((self.height, self.width, 4 if self.enable_alpha else 3), dtype=np.uint8)
        if not lib.GetFrameU8(self._ptr, out.ctypes.data_as(ctypes.c_void_p)):
            raise RuntimeError("GetFrameU8 failed: " + _lib.last_error())
        return out

    def frame_output_shape(self):
        """Shape of get_frame_u8()'s array: (H, W, ipp), or the flat YUV420P planes."""
        if lib.GetFrameFormat(self._ptr) == 1:
            return (self.width * self.height + 2 * (self.width // 2) * (self.height // 2),)
        return (self.height, self.width, 4 if self.enable_alpha else 3)

    def deliver_frame(self, dst: "HostBuffer") -> int:
        """Asynchronous copy of the last gathered frame output into the pinned
        host buffer `dst` (DeliverFrameU8), overlapped with the next frame;
        returns a ticket for wait_frame_delivered()."""
        n = int(np.prod(self.frame_output_shape()))
        if dst.nbytes < n:
            raise ValueError(f"deliver_frame: the host buffer holds {dst.nbytes} bytes, the frame {n}")
        t = lib.DeliverFrameU8(self._ptr, dst.ptr)
        if t < 0:
            raise RuntimeError("DeliverFrameU8 failed: " + _lib.last_error())
        return t

    def deliver_frame_bands(self, dst) -> int:
        """This rank's bands of its frame output (after its shard's frame --
        no gather) copied straight into their places in the host frame `dst`
        (a SharedHostBuffer every rank of the frame maps, or a HostBuffer in
        one process), asynchronously (DeliverFrameBands); returns a ticket
        for wait_frame_delivered().  The frame is whole once every rank's
        copy has landed."""
        n = int(np.prod(self.frame_output_shape()))
        if dst.nbytes < n:
            raise ValueError(f"deliver_frame_bands: the host buffer holds {dst.nbytes} bytes, the frame {n}")
        t = lib.DeliverFrameBands(self._ptr, dst.ptr)
        if t < 0:
            raise RuntimeError("DeliverFrameBands failed: " + _lib.last_error())
        return t

    def wait_frame_delivered(self, ticket: int):
        if not lib.WaitFrameDelivered(self._ptr, ticket):
            raise RuntimeError("WaitFrameDelivered failed: " + _lib.last_error())

    def set_frame_format(self, fmt: str):
        """Frame output of gather_frame_u8: "rgb" (the u8 image, cpp:52-57;
        default) or "yuv420p" (its YUV420P planes, the video encoder's input,
        written directly by the raster; even W and H)."""
        code = {"rgb": 0, "yuv420p": 1}[fmt]
        if not lib.SetFrameFormat(self._ptr, code):
            raise RuntimeError("SetFrameFormat failed: " + _lib.last_error())

    @staticmethod
    def gather_frame_u8_local(ctxs: typing.Sequence["RenderContext"], root: int = 0):
        """Testing: GatherFrameU8's packed band assembly for shards 0..n-1 of
        one process (ctxs[p] renders shard p of n), with device copies in
        place of the RCCL send/recv; the frame is assembled on ctxs[root]."""
        arr = (ctypes.c_void_p * len(ctxs))(*[c._ptr for c in ctxs])
        if not lib.GatherFrameU8Local(arr, len(ctxs), root):
            raise RuntimeError("GatherFrameU8Local failed: " + _lib.last_error())

    @staticmethod
    def gather_frame_u8_local_rccl(ctxs: typing.Sequence["RenderContext"], self_comm: "Comm", root: int = 0):
        """Testing: gather_frame_u8_local with the packs moved by RCCL
        send/recv pairs over a one-rank communicator of this process."""
        arr = (ctypes.c_void_p * len(ctxs))(*[c._ptr for c in ctxs])
        if not lib.GatherFrameU8LocalRccl(arr, len(ctxs), root, self_comm._ptr):
            raise RuntimeError("GatherFrameU8LocalRccl failed: " + _lib.last_error())

    def get_frame_yuv420p(self) -> np.ndarray:
        """YUV420P planes (Y, then U, then V) of the last gathered frame,
        converted on the GPU (GetFrameYUV420P; W and H even)."""
        n = self.width * self.height + 2 * (self.width // 2) * (self.height // 2)
        out = np.empty(n, dtype=np.uint8)
        if not lib.GetFrameYUV420P(self._ptr, out.ctypes.data_as(ctypes.c_void_p)):
            raise RuntimeError("GetFrameYUV420P failed: " + _lib.last_error())
        return out

    def gather_framebuffer(self, comm: "Comm", root: int = 0, with_depth: bool = True):
        """f64 framebuffer (+ depth) bands of every rank assembled on `root`
        (with_depth must be the same on every rank)."""
        if not lib.GatherFramebufferEx(self._ptr, comm._ptr, root, bool(with_depth)):
            raise RuntimeError("GatherFramebuffer failed: " + _lib.last_error())

    def last_raster_path(self) -> str:
        return {0: "none", 1: "order-free", 2: "ordered"}[lib.GetLastRasterPath(self._ptr)]

    def set_warm_binning(self, mode: int):
        """A TriangleBuffer drawn again under the binning key of its last
        validated draw bins in one pass into the kept tile ranges: 0 automatic
        (on), 1 on, 2 off (every draw counts, plans and emits)."""
        lib.SetWarmBinning(self._ptr, int(mode))

    def warm_batch_count(self) -> int:
        return lib.GetWarmBatchCount(self._ptr)

    def loose_batch_count(self) -> int:
        """Of the warm batches, those binned into the loose ranges of the
        schedule (the same buffer under a transform moved by <= 2 px)."""
        return lib.GetLooseBatchCount(self._ptr)

    def packed(self) -> "PackedCommands":
        """A packing front end of this context: its draw and state calls go
        to the library as one array per submit() (ExecuteCommands)."""
        return PackedCommands(self)

    def set_warm_fault_injection(self, mode: int):
        """Testing: a fault in the next warm batch (1 tile ranges overflow, 2
        the binning's token is withheld, 3 a workgroup's pairs are dropped, 4
        the binning is held back past the raster's token wait); the frame must
        stay exact and the failure be latched."""
        lib.SetWarmFaultInjection(self._ptr, int(mode))

    def warm_failure_count(self) -> int:
        return lib.GetWarmFailureCount(self._ptr)

    def set_force_ordered_raster(self, on: bool = True):
        lib.SetForceOrderedRaster(self._ptr, on)

    # ---- deferred command list (new) ---------------------
    def begin_commands(self):
        """Queue primitive draws until end_commands(): they then run as one
        launch, in order, with the immediate calls' exact results."""
        lib.BeginCommandList(self._ptr)

    def end_commands(self):
        lib.EndCommandList(self._ptr)

    def flush_commands(self):
        lib.FlushCommandList(self._ptr)

    def command_list_length(self) -> int:
        return lib.GetCommandListLength(self._ptr)

    def is_recording(self) -> bool:
        return bool(lib.IsRecordingCommands(self._ptr))

    class _Commands:
        def __init__(self, ctx):
            self.ctx = ctx

        def __enter__(self):
            self.ctx.begin_commands()
            return self.ctx

        def __exit__(self, *exc):
            self.ctx.end_commands()
            return False

    def commands(self):
        """`with ctx.commands(): ...` records the block's draws as one list."""
        return RenderContext._Commands(self)

    def set_coop_raster(self, mode: int):
        """k_vis variant (testing / A-B): 0 automatic, 1 wave-cooperative
        pass for large triangles, 2 lane-per-triangle only."""
        lib.SetCoopRaster(self._ptr, mode)

    def set_split_limits(self, split_at: int = 0, dslice: int = 0):
        """Testing / tuning: tiles of more than min(slice, split_at) pairs are
        split into slices of about `dslice` pairs (0: the defaults)."""
        lib.SetSplitLimits(self._ptr, split_at, dslice)

    def set_pair_capacity_override(self, pairs: int):
        """Testing: cap the visibility raster's (tile, triangle) list (0 = auto)."""
        lib.SetPairCapacityOverride(self._ptr, pairs)


class HostBuffer:
    """Pinned (page-locked) host memory from the library (AllocHostBuffer),
    the target of RenderContext.deliver_frame; `array(shape)` is a numpy view."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        self.ptr = lib.AllocHostBuffer(self.nbytes)
        if not self.ptr:
            raise MemoryError("AllocHostBuffer failed: " + _lib.last_error())

    def array(self, shape=None) -> np.ndarray:
        a = np.ctypeslib.as_array((ctypes.c_ubyte * self.nbytes).from_address(self.ptr))
        return a if shape is None else a[: int(np.prod(shape))].reshape(shape)

    def __del__(self):
        if getattr(self, "ptr", None):
            lib.FreeHostBuffer(self.ptr)
            self.ptr = None


class SharedHostBuffer:
    """Pinned host memory shared by the processes of a sharded frame (POSIX
    shared memory `name`, AllocSharedHostBuffer): every rank maps the same
    host frame and delivers its bands into it (deliver_frame_bands).  The
    creator (`owner=True`) removes the name when closed."""

    def __init__(self, name: str, nbytes: int, owner: bool = False):
        self.name, self.nbytes, self.owner = name, int(nbytes), owner
        self.ptr = lib.AllocSharedHostBuffer(name.encode(), self.nbytes)
        if not self.ptr:
            raise MemoryError("AllocSharedHostBuffer failed: " + _lib.last_error())

    def array(self, shape=None) -> np.ndarray:
        a = np.ctypeslib.as_array((ctypes.c_ubyte * self.nbytes).from_address(self.ptr))
        return a if shape is None else a[: int(np.prod(shape))].reshape(shape)

    def close(self):
        if getattr(self, "ptr", None):
            lib.FreeSharedHostBuffer(self.ptr, self.nbytes)
            self.ptr = None
            if self.owner:
                lib.UnlinkSharedHostBuffer(self.name.encode())

    def __del__(self):
        self.close()


class PackedCommands:
    """A RenderContext's draw and state calls packed on the host and submitted
    as ONE array per frame (ExecuteCommands) instead of one ctypes round trip
    per call -- the batching the reference's frame recorder
    MultiThreadedVideoRenderContextPreparer (Pybind:302-367) set out to do.

    It has the RenderContext methods a frame is drawn with (same names,
    arguments and results: every command runs through the same entry point, in
    order); anything else (get_transform, readbacks, triangles, ...) first
    submits what is packed and then goes to the context itself, so the two can
    be mixed freely.  Typical use: `cmds = ctx.packed()`, draw the frame through
    `cmds`, `cmds.submit()` (inside begin_commands()/flush_commands() the draws
    then run as one launch)."""

    __slots__ = ("_ctx", "_q", "_tex", "_tidx")

    def __init__(self, ctx: "RenderContext"):
        self._ctx = ctx
        self._q = []        # f64 words
        self._tex = []      # textures referenced by this submission (kept alive until it runs)
        self._tidx = {}

    def _t(self, tex) -> int:
        p = tex._ptr
        i = self._tidx.get(p)
        if i is None:
            i = self._tidx[p] = len(self._tex)
            self._tex.append(tex)
        return i

    def submit(self) -> int:
        """Runs the packed commands; returns how many ran."""
        if not self._q:
            return 0
        import array
        words = array.array("d", self._q)
        tex = (ctypes.c_void_p * max(len(self._tex), 1))(*[t._ptr for t in self._tex])
        n = lib.ExecuteCommands(self._ctx._ptr, words.buffer_info()[0], len(words), tex, len(self._tex))
        self._q.clear()
        self._tex.clear()
        self._tidx.clear()
        if n < 0:
            raise RuntimeError("ExecuteCommands failed: " + _lib.last_error())
        return n

    def __getattr__(self, name):
        self.submit()
        return getattr(self._ctx, name)

    # state (opcodes 0-10, ExecuteCommands)
    def save_state(self):
        self._q.append(0.0)

    def restore_state(self):
        self._q.append(1.0)

    def set_transform(self, a, b, c, d, e, f):
        self._q += (2.0, a, b, c, d, e, f)

    def apply_transform(self, a, b, c, d, e, f):
        self._q += (3.0, a, b, c, d, e, f)

    def scale(self, sx, sy):
        self._q += (4.0, sx, sy)

    def translate(self, tx, ty):
        self._q += (5.0, tx, ty)

    def rotate(self, angle):
        self._q += (6.0, angle)

    def rotate_degree(self, deg):
        self._q += (6.0, deg * math.pi / 180)   # (RenderContext.rotate_degree's expression)

    def set_color_transform(self, r, g, b, a):
        self._q += (7.0, r, g, b, a)

    def apply_color_transform(self, r, g, b, a):
        self._q += (8.0, r, g, b, a)

    def set_color(self, r, g, b, a):
        self._q += (9.0, r, g, b, a)

    def fill_color(self, r, g, b, a):
        self._q += (10.0, r, g, b, a)

    # draws (opcodes 11-18)
    def draw_texture(self, tex, x, y, w, h):
        self._q += (11.0, self._t(tex), x, y, w, h)

    def draw_splitted_texture(self, tex, x, y, width, height, u_start, u_end, v_start, v_end):
        self._q += (12.0, self._t(tex), x, y, width, height, u_start, u_end, v_start, v_end)

    def draw_rect(self, x, y, width, height, r, g, b, a):
        self._q += (13.0, x, y, width, height, r, g, b, a)

    def draw_line(self, x0, y0, x1, y1, width, r, g, b, a):
        self._q += (14.0, x0, y0, x1, y1, width, r, g, b, a)

    def draw_circle(self, x, y, radius, r, g, b, a):
        self._q += (15.0, x, y, radius, r, g, b, a)

    def draw_vertical_grd(self, x, y, width, height, top_r, top_g, top_b, top_a,
                          bottom_r, bottom_g, bottom_b, bottom_a):
        self._q += (16.0, x, y, width, height, top_r, top_g, top_b, top_a, bottom_r, bottom_g, bottom_b, bottom_a)

    def draw_vertical_mut_grd(self, x, y, width, height, steps):
        RenderContext.draw_vertical_mut_grd(self, x, y, width, height, steps)   # (bands -> draw_vertical_grd here)

    def set_pixel(self, x: int, y: int, r, g, b, a):
        self._q += (17.0, int(x), int(y), r, g, b, a)

    def apply_pixel(self, x: int, y: int, r, g, b, a):
        self._q += (18.0, int(x), int(y), r, g, b, a)


class RecordingRenderContext(RenderContext):
    """Counterpart of the reference's MultiThreadedVideoRenderContextPreparer
    (Pybind:302-367): it records each frame's draw calls and replays them.
    The reference's replay (`renderer`) is an unfinished stub and feeds a
    VideoCap (FFmpeg, out of scope); here the recording is the library's
    deferred command list and a frame's draws replay on the GPU as one launch
    at end_of_frame().  Transform / state calls apply immediately, as in the
    reference's `call_immediate_methods`."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.frames = 0
        self.begin_commands()

    def end_of_frame(self):
        self.flush_commands()
        self.frames += 1


class Texture:
    """Texels in HBM as f64, same interleaved layout as the framebuffer
    (cpp:318-354)."""

    def __init__(self, width: int, height: int, enableAlpha: bool, data: typing.ByteString,
                 is_uint8: bool = True):
        if width * height * (3 if not enableAlpha else 4) * (1 if is_uint8 else 8) != len(data):
            raise ValueError("data size not match")
        self.width = width
        self.height = height
        self.enableAlpha = enableAlpha
        self._can_release = False
        data = bytearray(data)
        if is_uint8:
            ptr = lib.CreateTextureUInt8(width, height, enableAlpha, (ctypes.c_byte * len(data)).from_buffer(data))
        else:
            ptr = lib.CreateTexture(width, height, enableAlpha, (ctypes.c_double * (len(data) // 8)).from_buffer(data))
        self._ptr = _check(ptr, "CreateTexture")
        self._can_release = True

    def __del__(self):
        if not getattr(self, "_can_release", False):
            return
        lib.DestroyTexture(self._ptr)
        self._can_release = False

    def _update_props(self):
        self.width = lib.GetTextureWidth(self._ptr)
        self.height = lib.GetTextureHeight(self._ptr)
        self.enableAlpha = lib.GetTextureEnableAlpha(self._ptr)

    def resample(self, width: int, height: int):
        return PtrCreatedTexture(_check(lib.ResampleTexture(self._ptr, width, height), "ResampleTexture"))

    def get_buffer_numpy(self) -> np.ndarray:
        ipp = 4 if self.enableAlpha else 3
        out = np.empty((self.height, self.width, ipp), dtype=np.float64)
        lib.GetTextureBuffer(self._ptr, _f64_ptr(out))
        return out

    @staticmethod
    def from_pilimg(img):
        from PIL import Image
        if not isinstance(img, Image.Image):
            raise TypeError("img must be a PIL.Image.Image")
        if img.mode not in ("RGB", "RGBA"):
            img = img.convert("RGBA")
        return Texture(img.width, img.height, img.mode == "RGBA", img.tobytes())

    @staticmethod
    def from_numpy(arr: np.ndarray) -> "Texture":
        """(H, W, 3|4) uint8 or float64 array -> Texture."""
        arr = np.ascontiguousarray(arr)
        h, w, c = arr.shape
        if arr.dtype == np.uint8:
            return Texture(w, h, c == 4, arr.tobytes())
        return Texture(w, h, c == 4, arr.astype(np.float64).tobytes(), is_uint8=False)


class PtrCreatedTexture(Texture):
    def __init__(self, ptr: int):
        self._ptr = ptr
        self._can_release = True
        self._update_props()


class TriangleBuffer:
    """Device-resident triangle soup (new): uploaded once, drawn per frame."""

    def __init__(self, xy, rgba, z=None, gouraud: typing.Optional[bool] = None):
        xy = np.ascontiguousarray(xy, dtype=np.float64).reshape(-1, 6)
        n = xy.shape[0]
        rgba = np.ascontiguousarray(rgba, dtype=np.float64)
        if gouraud is None:
            gouraud = rgba.size == 12 * n and n > 0
        rgba = rgba.reshape(n, 12 if gouraud else 4)
        if rgba.shape[1] != (12 if gouraud else 4):
            raise ValueError("rgba must hold 4 (flat) or 12 (Gouraud) values per triangle")
        zp = None
        if z is not None:
            z = np.ascontiguousarray(z, dtype=np.float64).reshape(n, 3)
            zp = _f64_ptr(z)
        self.n = n
        self.gouraud = bool(gouraud)
        self._can_release = False
        self._ptr = _check(lib.CreateTriangleBuffer(n, _f64_ptr(xy), zp, _f64_ptr(rgba), bool(gouraud)),
                           "CreateTriangleBuffer")
        self._can_release = True

    def __del__(self):
        if getattr(self, "_can_release", False):
            lib.DestroyTriangleBuffer(self._ptr)
            self._can_release = False


class Comm:
    """RCCL communicator (one rank per process/GPU) used to assemble sharded
    frames.  Rank 0 creates the id with Comm.unique_id() and every rank passes
    the same 128 bytes (e.g. via torch.distributed) to the constructor."""

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_ubyte * 128)()
        if not lib.GetCommUniqueId(buf):
            raise RuntimeError("GetCommUniqueId failed: " + _lib.last_error())
        return bytes(buf)

    def __init__(self, nranks: int, rank: int, uid: bytes):
        buf = (ctypes.c_ubyte * 128).from_buffer_copy(uid)
        self.nranks, self.rank = nranks, rank
        self._ptr = _check(lib.CreateComm(nranks, rank, buf), "CreateComm")

    def __del__(self):
        if getattr(self, "_ptr", None):
            lib.DestroyComm(self._ptr)
            self._ptr = None


class AudioClip:
    """Interleaved f64 samples in HBM (h:70-75); every operation is a kernel
    on the device's stream (csrc/nr_audio.hip).  Mirrors Pybind:503-660."""

    def __init__(self, sample_rate: int, channels: int, data: typing.Iterable[float]):
        data = np.ascontiguousarray(np.asarray(data, dtype=np.float64).reshape(-1))
        self._ptr = _check(lib.CreateAudioClipFromBuffer(sample_rate, channels, len(data) // max(channels, 1),
                                                         _f64_ptr(data)), "CreateAudioClipFromBuffer")
        self._update_props()

    def _update_props(self):
        self._sample_rate = lib.GetAudioClipSampleRate(self._ptr)
        self._channels = lib.GetAudioClipChannels(self._ptr)
        self._num_frames = lib.GetAudioClipNumFrames(self._ptr)

    @staticmethod
    def from_pydub_seg(seg):
        from pydub import AudioSegment   # absent in this image, as in the reference's demo path

        if not isinstance(seg, AudioSegment):
            raise TypeError("seg must be a pydub.AudioSegment")
        if seg.sample_width != 2:
            seg = seg.set_sample_width(2)
        data = seg.get_array_of_samples(array_type_override="h")
        return Int16CreatedAudioClip(seg.frame_rate, seg.channels, data)

    @staticmethod
    def slient(sample_rate: int, channels: int, num_frames: int):   # sic: the reference's name (Pybind:544)
        return PtrCreatedAudioClip(_check(lib.CreateSilentAudioClip(sample_rate, channels, num_frames),
                                          "CreateSilentAudioClip"))

    def clone(self):
        return PtrCreatedAudioClip(_check(lib.CloneAudioClip(self._ptr), "CloneAudioClip"))

    def resample(self, sample_rate: int, channels: int):
        lib.ApplyResampleAudioClip(self._ptr, sample_rate, channels)
        self._update_props()

    def resample_like(clip: "AudioClip", like: "AudioClip"):
        lib.ResampleAudioClipLike(clip._ptr, like._ptr)
        clip._update_props()

    @staticmethod
    def _raise(res: int):
        if res != 0:
            if res == -1:
                raise ValueError("target and source must have the same sample rate")
            if res == -2:
                raise ValueError("target and source must have the channels")
            raise ValueError(f"unknown error code: {res} {_lib.last_error()}")

    def overlay(target: "AudioClip", source: "AudioClip", start_time: typing.Union[int, float], *,
                time_unit: typing.Literal["frame", "second"] = "frame", auto_resample: bool = False):
        if time_unit not in ("frame", "second"):
            raise ValueError("time_unit must be 'frame' or 'second'")
        if time_unit == "frame":
            res = lib.OverlayAudioClip(target._ptr, source._ptr, int(start_time), auto_resample)
        else:
            res = lib.OverlayAudioClipSecond(target._ptr, source._ptr, float(start_time), auto_resample)
        AudioClip._raise(res)

    def overlay_many(target: "AudioClip", source: "AudioClip", start_times: typing.Sequence[typing.Union[int, float]],
                     *, time_unit: typing.Literal["frame", "second"] = "frame", auto_resample: bool = False):
        """New: the same result as ``for t in start_times: target.overlay(source, t, ...)``, in one launch."""
        if time_unit not in ("frame", "second"):
            raise ValueError("time_unit must be 'frame' or 'second'")
        if time_unit == "frame":
            st = np.ascontiguousarray(np.asarray(start_times, dtype=np.int64).reshape(-1))
            res = lib.OverlayAudioClipMany(target._ptr, source._ptr, st.ctypes.data_as(ctypes.c_void_p), len(st),
                                           auto_resample)
        else:
            st = np.ascontiguousarray(np.asarray(start_times, dtype=np.float64).reshape(-1))
            res = lib.OverlayAudioClipManySecond(target._ptr, source._ptr, _f64_ptr(st), len(st), auto_resample)
        AudioClip._raise(res)

    def save_as_wav(self):
        return Helpers.wappered_bytes_to_python(lib.SaveAudioClipAsWav(self._ptr))

    @property
    def duration(self):
        return lib.GetAudioClipDuration(self._ptr)

    def apply_volume_gain(self, gain: float):
        lib.ApplyVolumeGain(self._ptr, gain)

    def cut(self, start: typing.Union[int, float], end: typing.Union[int, float], *,
            time_unit: typing.Literal["frame", "second"] = "frame"):
        if time_unit not in ("frame", "second"):
            raise ValueError("time_unit must be 'frame' or 'second'")
        if time_unit == "frame":
            start, end = int(start), int(end)
        else:
            start, end = int(start * self._sample_rate), int(end * self._sample_rate)
        lib.ApplyCutAudioClip(self._ptr, start, end)
        self._update_props()

    def apply_speed(self, speed: float):
        lib.ApplySpeedAudioClip(self._ptr, speed)
        self._update_props()

    def to_numpy(self) -> np.ndarray:
        """New: the samples as a (frames, channels) float64 array."""
        self._update_props()
        out = np.empty((self._num_frames, self._channels), dtype=np.float64)
        if out.size:
            lib.GetAudioClipBuffer(self._ptr, _f64_ptr(out))
        return out

    def __del__(self):
        if getattr(self, "_ptr", None):
            lib.DestroyAudioClip(self._ptr)
            self._ptr = None


class Int16CreatedAudioClip(AudioClip):
    def __init__(self, sample_rate: int, channels: int, data: typing.Iterable[int]):
        data = np.ascontiguousarray(np.asarray(data, dtype=np.int16).reshape(-1))
        self._ptr = _check(lib.CreateAudioClipFromInt16Buffer(sample_rate, channels, len(data) // channels,
                                                              data.ctypes.data_as(ctypes.c_void_p)),
                           "CreateAudioClipFromInt16Buffer")
        self._update_props()


class PtrCreatedAudioClip(AudioClip):
    def __init__(self, ptr: int):
        self._ptr = ptr
        self._update_props()


def get_version():
    return lib.GetVersion()


def device_count() -> int:
    return lib.GetDeviceCount()


def set_device(device: int) -> bool:
    return lib.SetDevice(device)
