"""MI355X (gfx950) drop-in for libNativeCPURenderer's raster path.

Import the reference-compatible binding as
``from libnativecpurenderer_amd import libNativeCPURendererPybind as CPURenderer``.
"""
from ._lib import LIB_PATH  # noqa: F401

__all__ = ["LIB_PATH"]
