"""Loader for the in-tree native extension ``_C.so`` (gfx950 HIP kernels).

The extension is built by ``build.py`` (``__graft_entry__.build()`` does it for
the driver).  On a GPU box the HIP path *must* run our kernels: if the library
is missing we build it once, and if that fails we raise - there is no silent
fallback to ATen for GPU tensors.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_C = None


def load():
    global _C
    if _C is not None:
        return _C
    with _lock:
        if _C is not None:
            return _C
        here = os.path.dirname(os.path.abspath(__file__))
        so = os.path.join(here, "_C.so")
        if not os.path.exists(so) or os.environ.get("IMGCLS_REBUILD") == "1":
            from . import build as _build
            _build.build()
        import torch  # noqa: F401  (libtorch symbols must be loaded first)
        alt = os.environ.get("IMGCLS_EXT", "")
        if alt:  # same-box A/B of a compile-time variant (build.py --out NAME -DFLAG=...): load that file as _C
            import importlib.util as _ilu
            import sys
            path = alt if os.path.isabs(alt) else os.path.join(here, alt)
            spec = _ilu.spec_from_file_location(__package__ + "._C", path)
            _C = _ilu.module_from_spec(spec)
            spec.loader.exec_module(_C)
            sys.modules[__package__ + "._C"] = _C
            return _C
        _C = importlib.import_module(__package__ + "._C")
        return _C
