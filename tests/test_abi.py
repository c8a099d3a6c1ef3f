"""CPU checks of the drop-in boundary: the HIP library loads (no GPU needed
to load it), exports every symbol include/libNativeCPURenderer.h declares and
every render-path symbol of the reference ABI (h:83-152), and the Python
mirror exposes the reference binding's class/method surface.  No compute call
is made here."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "libNativeCPURenderer.h")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b([A-Z][A-Za-z0-9]*)\s*\(", text)
    return sorted(set(n for n in names if n not in ("RenderContext", "Texture", "TriangleBuffer")))


# The render-path entry points of the reference ABI (h:83-152) the reference's
# ctypes module binds (Pybind.py:51-440).  Media back-ends are out of scope.
REFERENCE_RENDER_SYMBOLS = [
    "GetBufferSize", "CreateRenderContext", "DestroyRenderContext", "ResizeRenderContext",
    "SaveContextState", "RestoreContextState", "GetBuffer", "GetBufferAsUInt8", "CreateTexture",
    "CreateTextureUInt8", "DestroyTexture", "CreateTextureFromRenderContext",
    "CreateTextureFromRenderContextShared", "SetTransform", "ApplyTransform", "Scale", "Translate",
    "Rotate", "TransformPoint", "GetTransform", "GetInverseTransform", "SetPixel", "ApplyPixel",
    "SetColorTransform", "ApplyColorTransform", "SetColor", "GetColor", "FillColor", "DrawTexture",
    "DrawRect", "DrawLine", "DrawCircle", "ResampleTexture", "GetTextureWidth", "GetTextureHeight",
    "GetTextureEnableAlpha", "GetVersion", "DrawVerticalGrd", "DrawSplittedTexture",
]


# The audio-clip entry points of the reference ABI (h:123-145) its AudioClip
# class binds (Pybind.py:503-660); SURVEY §8f-4.
REFERENCE_AUDIO_SYMBOLS = [
    "GetAudioClipBufferSizeFromData", "GetAudioClipBufferSize", "CreateAudioClipFromBuffer",
    "CreateAudioClipFromInt16Buffer", "CreateSilentAudioClip", "DestroyAudioClip", "CloneAudioClip",
    "ApplyResampleAudioClip", "ResampleAudioClipLike", "OverlayAudioClip", "OverlayAudioClipSecond",
    "SaveAudioClipAsWav", "GetAudioClipSampleRate", "GetAudioClipChannels", "GetAudioClipNumFrames",
    "GetAudioClipDuration", "GetWapperedBytesDataPtr", "GetWapperedBytesDataSize", "ApplyVolumeGain",
    "ApplyCutAudioClip", "ApplySpeedAudioClip",
]


def test_audio_symbols_declared_and_exported(hiplib):
    assert set(REFERENCE_AUDIO_SYMBOLS) <= set(header_symbols())
    for s in REFERENCE_AUDIO_SYMBOLS:
        assert hasattr(hiplib, s), s


@pytest.fixture(scope="module")
def hiplib():
    from libnativecpurenderer_amd import _lib
    return _lib.load()


def test_header_parses():
    syms = header_symbols()
    assert len(syms) > 60
    assert set(REFERENCE_RENDER_SYMBOLS) <= set(syms)


def test_library_exports_every_header_symbol(hiplib):
    missing = [s for s in header_symbols() if not hasattr(hiplib, s)]
    assert not missing, missing


def test_exports_are_unmangled_c_symbols():
    from libnativecpurenderer_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    defined = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for s in header_symbols():
        assert s in defined, s


def test_abi_table_matches_header(hiplib):
    from libnativecpurenderer_amd import _abi
    assert set(_abi.HIP_LIBRARY_ABI) == set(header_symbols())


def test_oracle_exports_reference_abi():
    import scenes
    from libnativecpurenderer_amd import _abi
    lib = ctypes.CDLL(scenes.build_oracle())
    for s in list(_abi.REFERENCE_ABI) + list(_abi.TRIANGLE_ABI):
        assert hasattr(lib, s), s


def test_python_surface_matches_reference_binding():
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    ref_ctx_methods = [
        "get_buffer_size", "get_buffer", "get_buffer_as_uint8", "fill_color", "draw_texture", "resize",
        "draw_splitted_texture", "apply_transform", "scale", "rotate", "translate", "rotate_degree",
        "save_state", "restore_state", "draw_line", "draw_rect", "get_transform", "get_inverse_transform",
        "apply_pixel", "draw_circle", "set_transform", "set_color_transform", "apply_color_transform",
        "set_pixel", "set_color", "get_color", "draw_vertical_grd", "draw_vertical_mut_grd", "as_texure",
        "as_texture_shared", "as_pilimg",
    ]
    for m in ref_ctx_methods:
        assert callable(getattr(R.RenderContext, m)), m
    for m in ["_update_props", "resample", "from_pilimg"]:
        assert callable(getattr(R.Texture, m)), m
    assert issubclass(R.PtrCreatedTexture, R.Texture)
    assert R.get_version() == 1


def test_no_cpu_fallback_without_device(hiplib):
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    if R.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(RuntimeError):
        R.RenderContext(8, 8, False)


def test_product_does_not_load_the_oracle():
    """The shipped package never loads or links the CPU restatement."""
    pkg = os.path.join(ROOT, "libnativecpurenderer_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(dirpath, f)).read()
                assert "liboracle" not in text and "oracle/build" not in text, f
                assert "import scenes" not in text, f
    out = subprocess.run(["ldd", os.path.join(pkg, "libNativeCPURenderer.so")], capture_output=True, text=True).stdout
    assert "oracle" not in out
