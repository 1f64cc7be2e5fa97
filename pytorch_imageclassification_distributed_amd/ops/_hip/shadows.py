"""bf16 weight shadows (KRSC and the transposed dgrad copy) and the MX-FP8 weight / activation copies
that the conv kernels read; the fused Adam kernel keeps registered shadows current.

Split out of ``ops/hip.py`` (the facade that re-exports every name here).
"""
from __future__ import annotations

import os
import weakref

import numpy as np
import torch

from .common import BF16, C, CL, _upload


# ---------------------------------------------------------------------------
# bf16 weight shadows
# ---------------------------------------------------------------------------
class _Shadow:
    # t: bf16 KRSC copy; tt: bf16 [Ci][T][Co] copy for dgrad (lazily, conv weights only).
    # stamp counts re-casts of t; tt is current when tt_stamp == stamp or the optimizer maintains it.
    __slots__ = ("t", "ptr", "version", "fused", "ref", "stamp", "tt", "tgeom", "tt_stamp", "tfused",
                 "mq", "ms", "m_stamp", "mfused")


_SHADOWS: dict = {}
_SHADOW_GEN = [0]


def _krsc_compatible(p: torch.Tensor) -> bool:
    if p.dim() != 4:
        return p.is_contiguous()
    return p.is_contiguous(memory_format=CL)


def weight_bf16(p: torch.Tensor) -> torch.Tensor:
    """bf16 copy of ``p`` in KRSC order ([Co][kh][kw][Ci] for conv weights).

    Refreshed when ``p`` changed outside the fused optimizer (version counter or storage moved):
    ``load_state_dict``, ``--pretrained`` into a live model, an EMA or any in-place edit bumps
    ``p._version``.  The fused Adam kernel writes the master and its shadows through raw pointers
    (no version bump), so a registered shadow stays current across steps without a re-cast, and a
    re-cast (``stamp`` += 1) invalidates the derived dgrad / MX copies even when the optimizer
    maintains them.
    """
    key = id(p)
    e = _SHADOWS.get(key)
    if e is not None and e.ref() is p and e.ptr == p.data_ptr() and e.version == p._version:
        return e.t
    if e is None or e.ref() is not p or e.t.numel() != p.numel():
        e = _Shadow()
        e.t = torch.empty(p.numel(), dtype=BF16, device=p.device)
        e.fused = False
        e.ref = weakref.ref(p)
        e.stamp, e.tt, e.tgeom, e.tt_stamp, e.tfused = 0, None, None, -1, False
        e.mq, e.ms, e.m_stamp, e.mfused = None, None, -1, False
        _SHADOWS[key] = e
        _SHADOW_GEN[0] += 1
    src = p.detach()
    # flatten in KRSC order: a free view for channels_last weights, a copy otherwise
    flat = src.permute(0, 2, 3, 1).reshape(-1) if src.dim() == 4 else src.reshape(-1)
    C.cast_bf16(flat, e.t)
    e.ptr = p.data_ptr()
    e.version = p._version
    e.stamp += 1
    return e.t


def weight_bf16_t(p: torch.Tensor, co: int, taps: int, ci: int) -> torch.Tensor:
    """bf16 copy of a KRSC conv weight transposed to [Ci][T][Co] (the dgrad B operand).

    Cached with the KRSC shadow; once registered with the fused Adam (``shadow_t_for_optimizer``)
    the optimizer rewrites it in its update pass (leaving ``stamp`` alone), so steady-state training
    never transposes; a re-cast of the KRSC shadow after an outside write makes it stale."""
    wb = weight_bf16(p)
    e = _SHADOWS[id(p)]
    if e.tt is not None and e.tgeom == (co, taps, ci) and e.tt_stamp == e.stamp:
        return e.tt
    if e.tt is None or e.tgeom != (co, taps, ci):
        e.tt = torch.empty(co * taps * ci, dtype=BF16, device=p.device)
        e.tgeom = (co, taps, ci)
        e.tfused = False
        _SHADOW_GEN[0] += 1  # the optimizer table picks the new copy up on its next step
    C.weight_t(wb, e.tt, co, taps, ci)
    e.tt_stamp = e.stamp
    return e.tt


def shadow_for_optimizer(p: torch.Tensor):
    """Shadow tensor the Adam kernel should rewrite for ``p`` (or None)."""
    e = _SHADOWS.get(id(p))
    if e is None or e.ref() is not p or not _krsc_compatible(p):
        return None
    e.fused = True
    return e.t


# ---------------------------------------------------------------------------
# MX-FP8 (forward convolutions, --dtype fp8)
# ---------------------------------------------------------------------------
FP8_FWD = os.environ.get("IMGCLS_FP8", "0") == "1"
FP8 = torch.float8_e4m3fn
_MXW_DT = np.dtype([("w", "<u8"), ("q", "<u8"), ("s", "<u8"), ("n", "<i8")])


def set_fp8(flag: bool = True) -> None:
    """MX-FP8 forward convolutions (e4m3 elements, E8M0 scale per 32 channels) wherever the input
    channel count is a multiple of 128; everything else (stem, 64-channel layers, backward) stays bf16."""
    global FP8_FWD
    FP8_FWD = bool(flag)


def _mx_tiles(jobs):
    return [(j, t) for j, (_w, _q, _s, n) in enumerate(jobs) for t in range(-(-n // 2048))]


def _mx_quant_weights(jobs, dev):
    arr = np.array(jobs, dtype=_MXW_DT)
    tiles = _mx_tiles(jobs)
    C.mx_quant_w(_upload(arr.view(np.uint8).copy(), dev), _upload(np.asarray(tiles, dtype=np.int32).reshape(-1), dev),
                 len(tiles))


def weight_mx(p: torch.Tensor):
    """(fp8 [Co*K], E8M0 [Co*K/32]) MX copy of a KRSC conv weight, quantised from the fp32 master.
    Kept current by the fused optimizer (one batched launch after Adam) once registered."""
    weight_bf16(p)  # creates / refreshes the shadow entry (version tracking lives there)
    e = _SHADOWS[id(p)]
    if e.mq is not None and e.m_stamp == e.stamp:
        return e.mq, e.ms
    if e.mq is None:
        if C.mx_wjob_bytes() != _MXW_DT.itemsize:
            raise RuntimeError("mx_quant_w: job record layout mismatch between Python and the kernel")
        e.mq = torch.empty(p.numel(), dtype=FP8, device=p.device)
        e.ms = torch.empty(p.numel() // 32, dtype=torch.uint8, device=p.device)
        e.mfused = False
        _SHADOW_GEN[0] += 1
    _mx_quant_weights([(p.data_ptr(), e.mq.data_ptr(), e.ms.data_ptr(), p.numel())], p.device)
    e.m_stamp = e.stamp
    return e.mq, e.ms


def shadow_mx_for_optimizer(p: torch.Tensor):
    e = _SHADOWS.get(id(p))
    if e is None or e.ref() is not p or e.mq is None or not _krsc_compatible(p):
        return None
    e.mfused = True
    return e.mq, e.ms


def act_mx(x: torch.Tensor):
    """MX-FP8 copy (fp8 [N*H*W*C], E8M0 [N*H*W*C/32]) of an NHWC bf16 activation, cached on the tensor
    so the several convolutions reading one activation quantise it once."""
    mx = getattr(x, "_imgcls_mx", None)
    if mx is not None and mx[2] == x._version:
        return mx[0], mx[1]
    n = x.numel()
    c = x.shape[1]
    q = torch.empty(n, dtype=FP8, device=x.device)
    sc = torch.empty(n // 32, dtype=torch.uint8, device=x.device)
    C.mx_quant_act(x, q, sc, n // c, c)
    x._imgcls_mx = (q, sc, x._version)
    return q, sc


def shadow_t_for_optimizer(p: torch.Tensor):
    """(transposed shadow, co, taps, ci) the Adam kernel should rewrite for ``p`` (or None)."""
    e = _SHADOWS.get(id(p))
    if e is None or e.ref() is not p or e.tt is None or not _krsc_compatible(p) or p.dim() != 4:
        return None
    e.tfused = True
    return (e.tt,) + e.tgeom


def shadow_generation() -> int:
    return _SHADOW_GEN[0]


def ensure_channels_last_weight(conv) -> None:
    w = conv.weight
    if w.dim() == 4 and not w.is_contiguous(memory_format=CL):
        w.data = w.data.contiguous(memory_format=CL)


# names this part owns (ops/hip.py re-exports them)
_OWNED = (
    'FP8', 'FP8_FWD', '_MXW_DT', '_SHADOWS', '_SHADOW_GEN', '_Shadow', '_krsc_compatible', '_mx_quant_weights',
    '_mx_tiles', 'act_mx', 'ensure_channels_last_weight', 'set_fp8', 'shadow_for_optimizer',
    'shadow_generation', 'shadow_mx_for_optimizer', 'shadow_t_for_optimizer', 'weight_bf16', 'weight_bf16_t',
    'weight_mx',
)
