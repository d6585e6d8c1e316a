"""Loader for the in-tree gfx950 kernel library (``_C/libdtfe_kernels.so``).

The library registers ``torch.ops.dtfe.*``.  It is loaded lazily the first
time a GPU op is needed.  On a GPU machine a missing or unloadable library is
a hard error (no silent eager fallback): ``require()`` raises.
"""
from __future__ import annotations

import os
import threading

import torch

_LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C")
# DTFE_KERNEL_LIB: load another build of the kernel library (csrc/build.py --ab: A/B of two code
# versions in one session on one GPU box)
KERNEL_LIB = os.environ.get("DTFE_KERNEL_LIB") or os.path.join(_LIB_DIR, "libdtfe_kernels.so")

_lock = threading.Lock()
_loaded = False
_err: Exception | None = None

# activation codes (csrc/kernels/common.h)
ACT_NONE, ACT_RELU, ACT_SIGMOID, ACT_TANH = 0, 1, 2, 3
ACT_CODES = {None: 0, "none": 0, "relu": 1, "sigmoid": 2, "tanh": 3}
# operand modes (csrc/kernels/gemm_core.h)
KMAJ, RMAJ = 0, 1
# optimizer kinds (csrc/kernels/optim.h)
OPT_SGD, OPT_MOMENTUM, OPT_ADAM, OPT_RMSPROP = 0, 1, 2, 3


def load(build_if_missing: bool = False) -> bool:
    """Load the kernel library; returns True on success."""
    global _loaded, _err
    with _lock:
        if _loaded:
            return True
        if not os.path.exists(KERNEL_LIB) and build_if_missing:
            from importlib import util

            spec = util.spec_from_file_location(
                "_dtfe_build", os.path.join(os.path.dirname(_LIB_DIR), "..", "csrc", "build.py"))
            mod = util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            mod.build("kernels")
        try:
            torch.ops.load_library(KERNEL_LIB)
            _loaded = True
            _err = None
        except Exception as e:  # noqa: BLE001 - reported by require()
            _err = e
        return _loaded


def require():
    """Return ``torch.ops.dtfe`` or raise if the native library is unavailable."""
    if not _loaded and not load():
        raise RuntimeError(
            f"dtfe: HIP kernel library not loadable ({KERNEL_LIB}): {_err!r}. "
            "Build it with `python csrc/build.py` (hipcc --offload-arch=gfx950).")
    return torch.ops.dtfe


def available() -> bool:
    return _loaded or load()
