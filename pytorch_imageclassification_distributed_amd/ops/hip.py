"""HIP path of the functional op layer: autograd Functions over the gfx950 kernels.

Tensor conventions on this path:
* activations: logical NCHW tensors in ``torch.channels_last`` memory format,
  bf16 - i.e. NHWC in memory, which is what every kernel in ``csrc/`` reads;
* conv weights: fp32 master parameters in channels_last (KRSC in memory); the
  kernels read a bf16 *shadow* of each weight that the fused Adam kernel
  rewrites after every step (see ``weight_bf16`` / ``engine.optim``);
* classifier features / logits: fp32 ``[N, C]``;
* BatchNorm statistics: fp32 partial sums produced by the conv epilogue,
  reduced in fp64; SyncBN exchanges the fp64 sums (one-shot xGMI peer kernel,
  ``parallel/peer.py``, or an RCCL all-reduce).

Every GPU op here is an in-tree kernel (``csrc/``): a missing extension raises, there is no
ATen / library-GEMM fallback on this path (the ATen path is ``--compute torch``).
"""
from __future__ import annotations

import sys
import types

from ._hip import adam, common, convbn, gemm, misc, pool, shadows, streams

_PARTS = {"common": common, "shadows": shadows, "gemm": gemm, "streams": streams, "pool": pool, "convbn": convbn,
          "misc": misc, "adam": adam}
# every public and private name of the parts, by owning module
_OWNER = {}
for _m in _PARTS.values():
    for _k in _m.__dict__.get("_OWNED", ()):
        _OWNER[_k] = _m
# Data (flags, counters, caches, tables) is read live from the owning part on every ``hip.X`` (tests and
# set_* functions rebind flags); functions and classes are copied here for plain attribute speed, except the
# ones scripts monkeypatch (scripts/conv_roofline.py, scripts/tune_random_choices.py).
_PATCHED = frozenset(("_conv_gemm", "_wgrad_launch", "_time_ms"))
_LATE = set(_PATCHED)
for _k, _m in _OWNER.items():
    _v = getattr(_m, _k)
    if isinstance(_v, (types.FunctionType, type)) and _k not in _PATCHED:
        globals()[_k] = _v
    else:
        _LATE.add(_k)


class _HipFacade(types.ModuleType):
    """``hip.X`` reads X from the module that owns it; ``hip.X = v`` rebinds it there, so the parts see
    flags set from outside (tests, scripts) exactly as the single module did."""

    def __getattr__(self, name):
        m = _OWNER.get(name)
        if m is None:
            raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
        return getattr(m, name)

    def __setattr__(self, name, value):
        m = _OWNER.get(name)
        if m is not None:
            setattr(m, name, value)
            if name in _LATE:
                return
        super().__setattr__(name, value)


sys.modules[__name__].__class__ = _HipFacade
