"""Import alias for the framework package.

The package lives in ``distributed-tensorflow-examples_amd/`` (a directory
name Python cannot import directly); ``import dtfe`` loads it from there and
registers it under the name ``dtfe`` so ``dtfe.models``, ``dtfe.parallel`` ...
resolve normally.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.abspath(__file__)), "distributed-tensorflow-examples_amd")
_spec = _ilu.spec_from_file_location("dtfe", _os.path.join(_PKG_DIR, "__init__.py"),
                                     submodule_search_locations=[_PKG_DIR])
_mod = _ilu.module_from_spec(_spec)
_sys.modules["dtfe"] = _mod
_spec.loader.exec_module(_mod)
