"""mxddp: an MI355X-native data-parallel training framework.

Capabilities of ``MyXiaoPao/distributed-training-dl`` (PyTorch single / DataParallel /
DDP trainers, TF2 single / Mirrored / MultiWorker, Chainer single / Parallel / MN)
re-designed as ONE PyTorch-ROCm trainer whose GPU hot path is hand-written HIP for
gfx950 (``mxddp/csrc``) and whose gradient exchange is an RCCL bucket reducer over xGMI.

The native extension is built in-tree (``python -m mxddp._build``).  On a GPU box every
op runs through it and fails loudly when it is missing; on CPU the same ops fall back to
plain PyTorch (BASELINE config 1, "single process on CPU").
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must be imported before the extension: shared HIP runtime)

__version__ = "0.1.0"

_C = None
_C_ERR: Exception | None = None


def native():
    """Return the native extension module, building it in-tree on first use if needed."""
    global _C, _C_ERR
    if _C is not None:
        return _C
    from . import _build

    if os.path.exists(_build.ext_path()) and _build.is_stale():
        # the in-tree module was built from different sources: rebuild, or refuse to run it
        if os.environ.get("MXDDP_NO_AUTOBUILD") or not os.path.exists(_build.HIPCC):
            raise ImportError(f"{_build.ext_path()} is stale (csrc changed since it was built); "
                              "run `python -m mxddp._build`")
        _build.build(verbose=True)
    try:
        _C = importlib.import_module("mxddp._C")
    except ImportError as e:  # not built yet
        if os.environ.get("MXDDP_NO_AUTOBUILD"):
            _C_ERR = e
            raise
        _build.build(verbose=True)
        _C = importlib.import_module("mxddp._C")
    return _C


def native_available() -> bool:
    try:
        native()
        return True
    except Exception:  # pragma: no cover - only on broken installs
        return False
