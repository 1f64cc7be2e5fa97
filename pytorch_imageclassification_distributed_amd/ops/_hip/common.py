"""Shared state of the HIP op layer: the extension handle, dtype / layout constants, deterministic mode,
BN-statistics pivots, per-device workspaces (zero page, statistics and partial-sum buffers) and small
tensor helpers.

Split out of ``ops/hip.py`` (the facade that re-exports every name here).
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.distributed as dist

from ... import _ext


C = _ext.load()

CL = torch.channels_last
BF16 = torch.bfloat16
ACT = {None: 0, "relu": 1, "silu": 2}
G_STATS = 64  # rotating partial rows for BN statistics atomics
DETERMINISTIC = os.environ.get("IMGCLS_DETERMINISTIC", "0") == "1"


def set_deterministic(flag: bool = True) -> None:
    """Bitwise-reproducible mode: every fp32 atomic site gets one contribution per address - BN partial
    rows >= producing blocks, no split-K (wgrad, head GEMMs), ordered column sums - and conv kernel choices
    come from the find-db or the shape heuristic, never from timing, so separate processes agree too.  Slower."""
    global DETERMINISTIC
    DETERMINISTIC = bool(flag)
    C.set_deterministic(DETERMINISTIC)


C.set_deterministic(DETERMINISTIC)


def set_force_div64(flag: bool = True) -> None:
    """Test hook: take the 64-bit index-division paths of the pool / depthwise / SE / GAP / stem-pool
    kernels (normally used only above 2^31 work items) at any size."""
    C.set_force_div64(bool(flag))


def stat_groups(rows: int) -> int:
    """Partial-sum rows for BN statistics over ``rows`` pixels: 64 rotating rows normally; in
    deterministic mode at least one per producing block (128-row conv tiles, <=1024 reduce blocks)."""
    return max(-(-rows // 128), 1024) if DETERMINISTIC else G_STATS
# BN statistics are summed about a per-channel pivot K = the BN's running mean (identical on every rank under
# SyncBN): sums of (x - K) and (x - K)^2, so var = S2/n - (S1/n)^2 cannot cancel at large |mean| / std once K
# tracks the batch mean (the shifted-data form of Chan's parallel combine; csrc/bn.hip).  The producer (conv
# epilogue, direct / stem kernels, bn_stats) and the finalize must use the same K: callers pass one tensor.
SHIFT_STATS = os.environ.get("IMGCLS_BN_SHIFT", "1") == "1"


def stat_shift(bn):
    """The pivot of ``bn``'s training statistics (its running mean), or None (pivot 0)."""
    rm = getattr(bn, "running_mean", None)
    if not (SHIFT_STATS and bn.training and getattr(bn, "track_running_stats", False) and rm is not None
            and rm.is_cuda and rm.dtype == torch.float32):
        return None
    return rm


FUSE_BN_BWD = os.environ.get("IMGCLS_FUSE_BN_BWD", "1") == "1"  # BN-backward reduce in the consumer's dgrad
FUSED_BWD_COUNT = [0]  # number of BN-backward reduces served by a conv epilogue (tests / diagnostics)


# ---------------------------------------------------------------------------
# per-device workspaces
# ---------------------------------------------------------------------------
class _Workspace:
    def __init__(self, dev):
        self.dev = dev
        self.stats = torch.zeros(0, dtype=torch.float32, device=dev)
        self.zero = torch.zeros(64, dtype=BF16, device=dev)  # zero page for padded LDS-DMA chunks
        self.parts: list = []  # zeroed partial-stat buffers for fused BN-backward reduces
        self.fin_ctr = torch.zeros(64, dtype=torch.int32, device=dev)  # bn_fin_apply's per-chunk block counters

    def take_part(self, c: int, groups: int = G_STATS) -> torch.Tensor:
        """A zeroed partial-sum buffer for a fused BN-backward reduce; handed back by ``give_part``
        after ``bn_partials`` has read (and re-zeroed) it, so the pool never needs a memset."""
        need = groups * 2 * c
        for i, b in enumerate(self.parts):
            if b.numel() >= need:
                return self.parts.pop(i)
        return torch.zeros(max(need, G_STATS * 2 * 2048), dtype=torch.float32, device=self.dev)

    def give_part(self, b: torch.Tensor) -> None:
        self.parts.append(b)

    def stats_buf(self, c: int, groups: int = G_STATS) -> torch.Tensor:
        need = groups * 2 * c
        if self.stats.numel() < need:
            # consumers re-zero what they read, so a fresh buffer only needs one memset
            self.stats = torch.zeros(max(need, G_STATS * 2 * 2048), dtype=torch.float32, device=self.dev)
        return self.stats


_WS: dict = {}


def ws(dev) -> _Workspace:
    key = (dev.type, dev.index)
    w = _WS.get(key)
    if w is None:
        w = _WS[key] = _Workspace(dev)
    return w


# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------
def _cl(x: torch.Tensor) -> torch.Tensor:
    return x if x.is_contiguous(memory_format=CL) else x.contiguous(memory_format=CL)


def _empty_cl(n, c, h, w, dev, dtype=BF16):
    return torch.empty((n, c, h, w), dtype=dtype, device=dev, memory_format=CL)


def _pad_tuple(conv, h, w):
    from ..functional import conv_padding
    return conv_padding(conv, h, w)


def _sync_group(bn):
    g = getattr(bn, "sync_group", None)
    if g is None or not dist.is_initialized() or dist.get_world_size(g) == 1:
        return None
    return g


def _upload(arr: np.ndarray, dev) -> torch.Tensor:
    # pinned + non_blocking: a pageable H2D copy would stall the host until the GPU drains
    return torch.from_numpy(arr).pin_memory().to(dev, non_blocking=True)


# names this part owns (ops/hip.py re-exports them)
_OWNED = (
    'ACT', 'BF16', 'C', 'CL', 'DETERMINISTIC', 'FUSED_BWD_COUNT', 'FUSE_BN_BWD', 'G_STATS', 'SHIFT_STATS',
    '_WS', '_Workspace', '_cl', '_empty_cl', '_pad_tuple', '_sync_group', '_upload', 'set_deterministic',
    'set_force_div64', 'stat_groups', 'stat_shift', 'ws',
)
