"""Loads the in-tree HIP library.  There is no CPU fallback: a missing or
unloadable libNativeCPURenderer.so raises, and so does a context creation on
a machine without a usable HIP device."""
from __future__ import annotations

import ctypes
import os

from . import _abi

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libNativeCPURenderer.so")

_lib = None


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is not built; run `make` or `python -c 'import __graft_entry__ as g; g.build()'`"
            )
        _lib = _abi.bind(ctypes.CDLL(LIB_PATH), _abi.HIP_LIBRARY_ABI)
    return _lib


def last_error() -> str:
    msg = load().GetLastErrorString()
    return msg.decode() if msg else ""


def clear_error() -> None:
    load().ClearLastError()
