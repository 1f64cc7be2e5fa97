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
# flags the tests / set_* functions rebind and functions scripts monkeypatch: read live from the owner
_LATE = frozenset((
    'CONCAT_INPLACE', 'CONV_FORCE_CFG', 'CONV_FORCE_FP8_CFG', 'CONV_STAGES', 'DEEP_BASE', 'DEEP_CONV',
    'DEEP_COUNT', 'DEEP_FORCE', 'DETERMINISTIC', 'DIRECT_BASE', 'DIRECT_CFGS', 'DIRECT_CONV', 'DIRECT_DGRAD',
    'DIRECT_FORCE', 'DW_LINK', 'FP8_FWD', 'FUSED_BWD_COUNT', 'FUSED_XA_BWD', 'FUSED_XA_BWD_COUNT',
    'FUSED_XA_BWD_N', 'FUSE_BN_BWD', 'FUSE_XA', 'FUSE_XF', 'GRAPH_SIDE', 'HALO_BASE', 'HALO_CONV', 'HALO_COUNT',
    'HALO_FORCE', 'HALO_TUNE', 'PEER_BN_MAX_C', 'POOL_CONV_SWAP', 'RELU_MASK', 'SE_FUSED', 'SE_LINK',
    'SHIFT_STATS', 'SKIP_WGRAD', 'STEM_DIRECT', 'STEM_POOL_FUSE', 'STEM_S2D', 'STEM_WGRAD_SIDE',
    'SYNCBN_EARLY_COUNT', 'TUNE_LOG', 'WGRAD_CANDIDATES', 'WGRAD_MIN_K', 'WGRAD_NARROW_TILES', 'WGRAD_STAGES',
    'WGRAD_STREAM', 'WGRAD_TARGET_BLOCKS', 'WGRAD_TUNE_LOG', 'WGRAD_WS', 'XA_COUNT', 'XA_MAX_REP',
    'XA_NARROW_OFF', 'XF_COUNT', 'XF_MAX_REP', '_ADAM_CHUNK', '_AFFINE_CACHE', '_CFGS', '_CU_COUNT',
    '_DEEP_CFGS', '_FP8_CFGS', '_HALO_CFGS', '_MXW_DT', '_ORDER_IDX', '_S2D_INDEX', '_SHADOWS', '_SHADOW_GEN',
    '_SIDE', '_STAGES_TUNED', '_TENSOR_DT', '_WGRAD_TUNED', '_WGRAD_WS', '_WS', '_WTJOB_DT', '_conv_gemm',
    '_time_ms', '_wgrad_launch',
))
for _k, _m in _OWNER.items():
    if _k not in _LATE:
        globals()[_k] = getattr(_m, _k)


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
