"""Loader for the CPU-side native runtime module ``_C/_dtfe_rt`` (pybind11).

Built by ``csrc/build.py`` (g++; no GPU needed).  If the module is missing it
is built on first use (a few seconds) - the runtime backs checkpoints, events
and the MNIST reader, which must work on CPU-only hosts too.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import sys
import threading

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_C = os.path.join(_PKG, "_C")
_lock = threading.Lock()
_mod = None


def _build():
    spec = importlib.util.spec_from_file_location("_dtfe_build", os.path.join(os.path.dirname(_PKG), "csrc",
                                                                              "build.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    b.build("rt")


def rt():
    global _mod
    with _lock:
        if _mod is not None:
            return _mod
        if _C not in sys.path:
            sys.path.insert(0, _C)
        try:
            _mod = importlib.import_module("_dtfe_rt")
        except ImportError:
            _build()
            importlib.invalidate_caches()
            _mod = importlib.import_module("_dtfe_rt")
        return _mod
