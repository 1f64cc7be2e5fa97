"""Weight gradients on a side stream: the stream registry, the fork / join around each launch and the
all-reduce stream the gradient reducer uses.

Split out of ``ops/hip.py`` (the facade that re-exports every name here).
"""
from __future__ import annotations

import os

import torch

from ..grad_arena import arena_slot, grad_buffer
from . import gemm as _gemm
from .common import C
from .gemm import ConvGeom, _wgrad_plan


# ---------------------------------------------------------------------------
# weight gradients on a side stream
# ---------------------------------------------------------------------------
# A weight gradient is off the backward critical path: only the optimizer (and the bucket all-reduce)
# read it, while the next layer's backward needs only the data gradient.  Each conv's wgrad GEMM is
# therefore enqueued on a second HIP stream behind an event on the compute stream, so it runs beside the
# dgrad -> BN-backward chain of the layers below (filling the last partial wave of a 1-2 wave launch, and
# pairing compute-bound wgrad tiles with bandwidth-bound BN kernels on the same CUs).  Only gradients
# that land in an armed arena slot go there (autograd adopts the slot without reading it); the compute
# stream waits for the side stream when backward ends (an engine callback), and the reducer issues each
# bucket's all-reduce behind both streams.  IMGCLS_WGRAD_STREAM=0 keeps everything on one stream.
WGRAD_STREAM = os.environ.get("IMGCLS_WGRAD_STREAM", "1") == "1"
# inside a HIP-graph capture the weight gradients stay on the capturing stream: a two-stream capture
# (event fork / join edges) replays 2x slower than the single-stream one on this ROCm runtime
# (Inception-v3 b128: 3303 vs 6523 img/s, profiles/history/r3g_hip_graph_modes.txt); IMGCLS_GRAPH_SIDE=1 forks
GRAPH_SIDE = os.environ.get("IMGCLS_GRAPH_SIDE", "0") == "1"
_SIDE: dict = {}  # device index -> _SideStream
# < 1: the side stream's kernels may occupy only this fraction of the CUs (a CU-masked HIP stream, k of every 8
# CUs of each XCD whichever way the driver numbers them), so a long weight-gradient wave cannot hold CUs the
# compute stream's next launch needs; 1 (default): all CUs, the compute stream wins only by queue priority
WGRAD_CU_FRAC = float(os.environ.get("IMGCLS_WGRAD_CU_FRAC", "1"))


def cu_mask_words(n_cu: int, frac: float) -> list:
    """32-bit CU mask words enabling round(8 * frac) of every 8 CUs: CU i is on when (i // 8 + i) % 8 < k, which
    keeps k of 8 per XCD for XCD-major (i // 32) and XCD-interleaved (i % 8) numbering alike."""
    k = max(1, min(8, round(8 * frac)))
    words = [0] * (-(-n_cu // 32))
    for i in range(n_cu):
        if (i // 8 + i) % 8 < k:
            words[i // 32] |= 1 << (i % 32)
    return words


class _SideStream:
    __slots__ = ("stream", "joins", "handle", "ws")

    def __init__(self, dev):
        if WGRAD_CU_FRAC < 1:
            n_cu = torch.cuda.get_device_properties(dev).multi_processor_count
            ptr = C.cu_mask_stream(dev.index, cu_mask_words(n_cu, WGRAD_CU_FRAC))
            self.stream = torch.cuda.ExternalStream(ptr, device=dev)
        else:
            self.stream = torch.cuda.Stream(device=dev)
        self.joins = set()  # compute streams that must wait for this stream when backward ends
        self.handle = self.stream.cuda_stream  # raw hipStream_t for launchers that fork to it themselves
        self.ws = None  # split-K workspace of the wgrad launches on this stream


def side_stream(dev):
    """The weight-gradient stream of ``dev``, or None (disabled, CPU, or inside a graph capture with
    IMGCLS_GRAPH_SIDE=0)."""
    if not WGRAD_STREAM or dev.type != "cuda" or (not GRAPH_SIDE and torch.cuda.is_current_stream_capturing()):
        return None
    s = _SIDE.get(dev.index)
    if s is None:
        s = _SIDE[dev.index] = _SideStream(dev)
    return s


def join_side_streams() -> None:
    """Make every compute stream that handed work to a side stream wait for it (no host sync)."""
    from ...parallel import comm_timer
    for s in _SIDE.values():
        for main in s.joins:
            comm_timer.mark("compute_end", main)
            main.wait_stream(s.stream)
            comm_timer.mark("side_joined", main)
        s.joins.clear()


def _on_side(dev, launch, *keep):
    """Run ``launch()`` on the side stream of ``dev`` behind the current stream's work so far; the
    tensors in ``keep`` stay allocated until the side stream is done with them."""
    s = side_stream(dev)
    if s is None:
        launch()
        return
    main = torch.cuda.current_stream(dev)
    if not s.joins:
        # first side launch of this backward: join when the engine finishes the whole graph
        torch.autograd.Variable._execution_engine.queue_callback(join_side_streams)
    s.joins.add(main)
    s.stream.wait_stream(main)
    with torch.cuda.stream(s.stream):
        launch()
    for t in keep:
        t.record_stream(s.stream)


def comm_stream(dev):
    """Stream to issue a gradient all-reduce on: the side stream after it has waited for the compute
    stream (so the collective follows every gradient of both), or None for the current stream."""
    s = _SIDE.get(dev.index) if dev.type == "cuda" else None
    if s is None or not s.joins:
        return None
    s.stream.wait_stream(torch.cuda.current_stream(dev))
    return s.stream


# 1: the input layer's weight gradient joins the side stream like every other (the round-2 placement)
STEM_WGRAD_SIDE = os.environ.get("IMGCLS_STEM_WGRAD_SIDE", "0") == "1"


def conv_wgrad_raw(dy, x, w_param, g: ConvGeom, xa=None, xf=None):
    dev = dy.device
    m = g.N * g.OH * g.OW
    ntot = g.T * g.Cx
    kps, splits, stages = _wgrad_plan(g, dy, x, m, ntot, xa, xf)
    if (xa is not None or xf is not None) and g.Cx != g.Ci:
        raise RuntimeError("fused BN wgrad: padded input channels")
    if g.Cx == g.Ci:
        dw = arena_slot(w_param)
        if dw is not None:
            s = side_stream(dev)
            if s is None:
                _gemm._wgrad_launch(dy, x, dw, g, m, ntot, kps, splits, stages, xa=xa, xf=xf)
                return dw
            if not s.joins:  # first side launch of this backward: join when the engine finishes
                torch.autograd.Variable._execution_engine.queue_callback(join_side_streams)
            s.joins.add(torch.cuda.current_stream(dev))
            _gemm._wgrad_launch(dy, x, dw, g, m, ntot, kps, splits, stages, side=s, xa=xa, xf=xf)
            return dw
        dw = grad_buffer(w_param)
        _gemm._wgrad_launch(dy, x, dw, g, m, ntot, kps, splits, stages, xa=xa, xf=xf)
        return dw
    full = torch.zeros(g.Co * ntot, dtype=torch.float32, device=dev)
    dw = arena_slot(w_param)
    if dw is not None:
        # padded input channels = the network's input layer, the last weight gradient of backward: on the
        # compute stream (idle by then) it runs beside the side stream's backlog instead of behind it - the
        # ResNet-50 b1024 stem wgrad is ~0.7 ms of the step tail (profiles/history/r5e_conv_roofline_b1024.txt)
        if STEM_WGRAD_SIDE:
            def launch():
                _gemm._wgrad_launch(dy, x, full, g, m, ntot, kps, splits, stages)
                C.grad_unpad(full, dw, g.Co * g.T, g.Cx, g.Ci)
            _on_side(dev, launch, dy, x, full)
            return dw
        _gemm._wgrad_launch(dy, x, full, g, m, ntot, kps, splits, stages)
        C.grad_unpad(full, dw, g.Co * g.T, g.Cx, g.Ci)
        return dw
    _gemm._wgrad_launch(dy, x, full, g, m, ntot, kps, splits, stages)
    dw = grad_buffer(w_param, zero=False)
    C.grad_unpad(full, dw, g.Co * g.T, g.Cx, g.Ci)
    return dw


# names this part owns (ops/hip.py re-exports them)
_OWNED = (
    'GRAPH_SIDE', 'STEM_WGRAD_SIDE', 'WGRAD_CU_FRAC', 'WGRAD_STREAM', '_SIDE', '_SideStream', '_on_side',
    'comm_stream', 'conv_wgrad_raw', 'cu_mask_words', 'join_side_streams', 'side_stream',
)
