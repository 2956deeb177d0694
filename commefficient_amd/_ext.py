"""Loader for the native extension (``_C.so``: HIP gfx950 kernels + CPU kernels).

The extension registers ``torch.ops.commeff.*``.  There is deliberately no
pure-PyTorch fallback: if the library is missing the import fails loudly
(on a GPU box a silent eager fallback would hide that native code is not
running).  Set ``COMMEFF_AUTOBUILD=1`` to build it in-tree on first import.
"""
from __future__ import annotations

import os
import threading

import torch

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_C.so")
# A/B measurements only: load another build of the same sources instead
_LIB = os.environ.get("COMMEFF_LIB") or _LIB
_lock = threading.Lock()
_loaded = False


def load() -> None:
    global _loaded
    if _loaded:
        return
    with _lock:
        if _loaded:
            return
        if not os.path.exists(_LIB):
            if os.environ.get("COMMEFF_AUTOBUILD", "0") == "1":
                from . import build
                build.build()
            else:
                raise ImportError(
                    f"commefficient_amd native extension not built ({_LIB} missing). "
                    "Run `python -m commefficient_amd.build` (hipcc --offload-arch=gfx950).")
        torch.ops.load_library(_LIB)
        _loaded = True


def ops():
    load()
    return torch.ops.commeff


def library_path() -> str:
    return _LIB
