"""Pooling autograd Functions (max / average / global average) and the channel-slice stride helper.

Split out of ``ops/hip.py`` (the facade that re-exports every name here).
"""
from __future__ import annotations

import torch

from .common import C, _cl, _empty_cl


# ---------------------------------------------------------------------------
# pooling
# ---------------------------------------------------------------------------
def _pool_args(k, s, p):
    k = (k, k) if isinstance(k, int) else tuple(k)
    s = (s, s) if isinstance(s, int) else tuple(s)
    p = (p, p) if isinstance(p, int) else tuple(p)
    return k, s, p


class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, slot=None):
        n, c, h, w = x.shape
        oh = (h + 2 * p[0] - k[0]) // s[0] + 1
        ow = (w + 2 * p[1] - k[1]) // s[1] + 1
        y = _empty_cl(n, c, oh, ow, x.device)
        idx = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=x.device)
        C.maxpool_fwd(x, y, idx, n, h, w, c, oh, ow, k[0], k[1], s[0], s[1], p[0], p[1])
        ctx.geo = (n, h, w, c, oh, ow, k, s, p)
        ctx.slot = slot
        ctx.save_for_backward(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        n, h, w, c, oh, ow, k, s, p = ctx.geo
        dx = _empty_cl(n, c, h, w, dy.device)
        C.maxpool_bwd(_cl(dy), idx, dx, n, h, w, c, oh, ow, k[0], k[1], s[0], s[1], p[0], p[1])
        if ctx.slot is not None:
            dx = ctx.slot.deliver(dx)
        return dx, None, None, None, None


def max_pool2d(x, kernel_size, stride, padding=0, slot=None):
    k, s, p = _pool_args(kernel_size, stride, padding)
    return MaxPoolFn.apply(_cl(x), k, s, p, slot)


class AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, slot=None):
        n, c, h, w = x.shape
        oh = (h + 2 * p[0] - k[0]) // s[0] + 1
        ow = (w + 2 * p[1] - k[1]) // s[1] + 1
        y = _empty_cl(n, c, oh, ow, x.device)
        C.avgpool_fwd(x, y, n, h, w, c, oh, ow, k[0], k[1], s[0], s[1], p[0], p[1])
        ctx.geo = (n, h, w, c, oh, ow, k, s, p)
        ctx.slot = slot
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c, oh, ow, k, s, p = ctx.geo
        dx = _empty_cl(n, c, h, w, dy.device)
        C.avgpool_bwd(_cl(dy), dx, n, h, w, c, oh, ow, k[0], k[1], s[0], s[1], p[0], p[1])
        if ctx.slot is not None:
            dx = ctx.slot.deliver(dx)
        return dx, None, None, None, None


def avg_pool2d(x, kernel_size, stride, padding=0, slot=None):
    k, s, p = _pool_args(kernel_size, stride, padding)
    return AvgPoolFn.apply(_cl(x), k, s, p, slot)


class GapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        n, c, h, w = x.shape
        y = torch.empty((n, c), dtype=torch.float32, device=x.device)
        C.gap_fwd(x, y, n, h * w, c)
        ctx.geo = (n, c, h, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, c, h, w = ctx.geo
        dx = _empty_cl(n, c, h, w, dy.device)
        C.gap_bwd(dy.contiguous().float(), dx, n, h * w, c)
        return dx


def global_avg_pool(x):
    return GapFn.apply(_cl(x))


def channel_slice_stride(t) -> int:
    """Row stride (channels) when ``t`` is a channel slice of a wider channels-last tensor (a concat
    output's per-branch gradient), else 0."""
    if t.dim() != 4 or t.stride(1) != 1:
        return 0
    n, c, h, w = t.shape
    ld = t.stride(3)
    if ld == c or ld % 8 or c % 8 or t.stride(2) != w * ld or (n > 1 and t.stride(0) != h * w * ld):
        return 0
    return ld if t.data_ptr() % 16 == 0 else 0


# names this part owns (ops/hip.py re-exports them)
_OWNED = (
    'AvgPoolFn', 'GapFn', 'MaxPoolFn', '_pool_args', 'avg_pool2d', 'channel_slice_stride', 'global_avg_pool',
    'max_pool2d',
)
