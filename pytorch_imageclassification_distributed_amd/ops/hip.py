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

import math
import os
import weakref

import numpy as np
import torch
import torch.distributed as dist

from .. import _ext
from ..parallel.peer import PeerWork, peer_channel, side_stream as peer_side_stream
from ..parallel.peer import stats_all_reduce_, stats_all_reduce_async
from .grad_arena import arena_slot, grad_buffer

C = _ext.load()

CL = torch.channels_last
BF16 = torch.bfloat16
ACT = {None: 0, "relu": 1, "silu": 2}
G_STATS = 64  # rotating partial rows for BN statistics atomics
DETERMINISTIC = os.environ.get("IMGCLS_DETERMINISTIC", "0") == "1"


def set_deterministic(flag: bool = True) -> None:
    """Bitwise-reproducible mode: every fp32 atomic site gets one contribution per address - BN partial
    rows >= producing blocks, no split-K (wgrad, head GEMMs), ordered column sums.  Slower."""
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


# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------
def _cl(x: torch.Tensor) -> torch.Tensor:
    return x if x.is_contiguous(memory_format=CL) else x.contiguous(memory_format=CL)


def _empty_cl(n, c, h, w, dev, dtype=BF16):
    return torch.empty((n, c, h, w), dtype=dtype, device=dev, memory_format=CL)


def _pad_tuple(conv, h, w):
    from .functional import conv_padding
    return conv_padding(conv, h, w)


def _sync_group(bn):
    g = getattr(bn, "sync_group", None)
    if g is None or not dist.is_initialized() or dist.get_world_size(g) == 1:
        return None
    return g


# ---------------------------------------------------------------------------
# convolution (implicit GEMM on MFMA)
# ---------------------------------------------------------------------------
class ConvGeom:
    __slots__ = ("N", "Ci", "Cx", "H", "W", "Co", "kh", "kw", "sh", "sw", "dil", "pt", "pb", "pl", "pr",
                 "OH", "OW", "T", "taps", "phases")

    def __init__(self, x, conv):
        self.taps = self.phases = None  # memoised _fwd_taps / _dgrad_phases (host time per launch)
        self.N, self.Cx, self.H, self.W = x.shape
        self.Co, self.Ci, self.kh, self.kw = conv.weight.shape
        self.sh, self.sw = conv.stride
        self.dil = conv.dilation[0]
        if conv.dilation[0] != conv.dilation[1]:
            raise NotImplementedError("anisotropic dilation")
        self.pt, self.pb, self.pl, self.pr = _pad_tuple(conv, self.H, self.W)
        self.OH = (self.H + self.pt + self.pb - self.dil * (self.kh - 1) - 1) // self.sh + 1
        self.OW = (self.W + self.pl + self.pr - self.dil * (self.kw - 1) - 1) // self.sw + 1
        self.T = self.kh * self.kw


def conv_geom(x, conv) -> ConvGeom:
    """``ConvGeom(x, conv)`` memoised on the module per input shape: the geometry, its tap table and its
    dgrad phases are computed once, not on every launch (host time: Inception-v3 runs ~95 convs a step)."""
    cache = conv.__dict__.get("_imgcls_geom")
    if cache is None:
        cache = conv.__dict__["_imgcls_geom"] = {}
    g = cache.get(x.shape)
    if g is None:
        g = cache[x.shape] = ConvGeom(x, conv)
    return g


def _fwd_taps(g: ConvGeom):
    if g.taps is not None:
        return g.taps
    dh, dw, tb = [], [], []
    for r in range(g.kh):
        for c in range(g.kw):
            dh.append(r * g.dil - g.pt)
            dw.append(c * g.dil - g.pl)
            tb.append(r * g.kw + c)
    g.taps = (tuple(dh), tuple(dw), tuple(tb))
    return g.taps


def _dgrad_phases(g: ConvGeom):
    """Sub-pixel decomposition of the transposed convolution (one GEMM per phase)."""
    if g.phases is not None:
        return g.phases
    out = []
    for ph in range(g.sh):
        for pw in range(g.sw):
            dh, dw, tb = [], [], []
            for r in range(g.kh):
                a = ph + g.pt - r * g.dil
                if a % g.sh:
                    continue
                for c in range(g.kw):
                    b = pw + g.pl - c * g.dil
                    if b % g.sw:
                        continue
                    dh.append(a // g.sh)
                    dw.append(b // g.sw)
                    tb.append(r * g.kw + c)
            gh = (g.H - ph + g.sh - 1) // g.sh
            gw = (g.W - pw + g.sw - 1) // g.sw
            out.append((ph, pw, gh, gw, tuple(dh), tuple(dw), tuple(tb)))
    g.phases = tuple(out)
    return g.phases


def _weight_for_input(w_param, cx):
    """bf16 KRSC weight, zero-padded along Ci when the input carries padded channels (stem)."""
    wb = weight_bf16(w_param)
    co, ci, kh, kw = w_param.shape
    if cx == ci:
        return wb
    out = torch.empty(co * kh * kw * cx, dtype=BF16, device=w_param.device)
    C.weight_pad(wb, out, co * kh * kw, ci, cx)
    return out


def _time_ms(run, reps: int = 3, trials: int = 3) -> float:
    """Best-of-``trials`` mean time of ``reps`` back-to-back launches (after one warm launch):
    the minimum is robust to the occasional preempted trial that made single-shot choices noisy."""
    run()
    best = float("inf")
    for _ in range(trials):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            run()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) / reps)
    return best


CONV_STAGES = os.environ.get("IMGCLS_CONV_STAGES", "auto")  # auto (timed per shape) | 0 (heuristic) | 1 | 2
_STAGES_TUNED: dict = {}


def save_tuning(path: str) -> int:
    """Write the per-shape kernel choices found so far (conv fwd/dgrad configurations, wgrad split and
    variant) to a JSON "find-db"; returns the entry count.  ``load_tuning`` seeds a later process with
    them, so its choices are the same (and it skips the timing) - like a conv-algorithm find-db."""
    import json
    db = {"conv": [[repr(k), list(v)] for k, v in _STAGES_TUNED.items()],
          "wgrad": [[repr(k), list(v)] for k, v in _WGRAD_TUNED.items()]}
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    with open(path, "w") as f:
        json.dump(db, f, indent=0)
    return len(db["conv"]) + len(db["wgrad"])


def load_tuning(path: str) -> int:
    """Seed the tuning caches from a ``save_tuning`` file (entries already present win; entries naming a
    configuration this build does not have are skipped).  Keys are parsed with ast.literal_eval."""
    import ast
    import json
    try:
        with open(path) as f:
            db = json.load(f)
    except (OSError, ValueError):
        return 0
    n = 0
    ncfg, nfp8 = len(conv_cfgs()), len(conv_fp8_cfgs())
    for ks, v in db.get("conv", []):
        try:
            k, v = ast.literal_eval(ks), tuple(int(x) for x in v)
        except (ValueError, SyntaxError, TypeError):
            continue
        fp8 = bool(k[10]) if len(k) > 10 else False
        if v[2] >= DEEP_BASE:
            ok = not fp8 and v[2] - DEEP_BASE < len(conv_deep_cfgs()) and len(v) == 3
        elif v[2] >= HALO_BASE:
            ok = not fp8 and v[2] - HALO_BASE < len(conv_halo_cfgs()) and len(v) == 3
        else:
            ok = (v[2] - DIRECT_BASE in DIRECT_CFGS if v[2] >= DIRECT_BASE else
                  v[2] < (nfp8 if fp8 else ncfg)) and len(v) == 3
        if ok and k not in _STAGES_TUNED:
            _STAGES_TUNED[k] = v
            n += 1
    for ks, v in db.get("wgrad", []):
        try:
            k, v = ast.literal_eval(ks), tuple(int(x) for x in v)
        except (ValueError, SyntaxError, TypeError):
            continue
        if len(v) == 2 and 1 <= v[1] <= 12 and v[0] > 0 and k not in _WGRAD_TUNED:
            _WGRAD_TUNED[k] = v
            n += 1
    return n
CONV_FORCE_CFG = None  # (stages, tile_n, cfg) for every bf16 fwd/dgrad launch (tests)
CONV_FORCE_FP8_CFG = None  # (stages, tile_n, cfg) for every MX-FP8 forward launch (tests)
TUNE_LOG: list = []  # (M, Ncols, K, {cfg: ms}) per tuned geometry (benchmarks/conv_bench.py prints it)


def _conv_gemm(A, B, out, stats, bias, geo, dh, dw, tb, zero, addend=None, bwd=(None, None, None, None, 0, 1),
               groups=G_STATS, scales=(None, None), xa=None, shift=None, xf=None, mask=None):
    """One implicit-GEMM launch.  The kernel configuration - LDS-DMA ring depth (1 = high occupancy,
    2 / 3 = pipelined) x output-channel tile (64 / 128 / 256: more tiles balance 256 CUs better on
    small layers) x pixel tile (128 rows on 4 waves, or 256 rows on 8 waves) - is chosen once per
    GEMM geometry by timing the candidates on scratch outputs (a conv-algorithm "find" step).
    ``xa`` = (y, coef [3][CA]): A holds a BN's pre-elementwise gradient dz and the kernel applies the
    BN backward's elementwise map on its operand loads (1x1 stride-1 geometry; ``XaLink``).
    ``xf`` = (coef, act): A holds a BN's input y and the kernel applies act(bn(y)) on its operand loads
    (``XfHold``)."""
    xa3 = (xa[0], xa[1], None) if xa is not None else (None, None, None)
    xf2 = (xf[0], xf[1]) if xf is not None else (None, 0)
    fused = xa is not None or xf is not None
    if DIRECT_FORCE is not None and not fused and \
            _direct_geom(geo, dh, dw, tb, out, bias, addend, bwd, scales) is not None:
        cfg = (0, 0, DIRECT_BASE + DIRECT_FORCE)  # (tests) every eligible launch on this direct variant
    elif DEEP_FORCE is not None and not fused and scales[0] is None and _deep_ok(geo, dh, dw):
        cfg = (0, 0, DEEP_BASE + DEEP_FORCE)  # (tests) every eligible launch on this prefetch-depth-2 variant
    elif HALO_FORCE is not None and not fused and scales[0] is None and \
            _halo_ok(geo, dh, dw, *conv_halo_cfgs()[HALO_FORCE][::5]):
        cfg = (0, 0, HALO_BASE + HALO_FORCE)  # (tests) every eligible launch on this halo variant
    elif CONV_FORCE_CFG is not None and scales[0] is None and (not fused or C.conv_cfg_has_xa(CONV_FORCE_CFG[2])):
        cfg = CONV_FORCE_CFG
    elif CONV_FORCE_FP8_CFG is not None and scales[0] is not None:
        cfg = CONV_FORCE_FP8_CFG
    elif CONV_STAGES != "auto":
        cfg = (int(CONV_STAGES), 0, -1)
    else:
        key = (tuple(geo), out.shape[1], tuple(dh), tuple(dw), stats is not None, bias is not None,
               addend is not None, bwd[0] is not None, bwd[1] is not None, bwd[4], scales[0] is not None,
               DIRECT_CONV) + ((True,) if xa is not None else ()) + (("xf",) if xf is not None else ())
        cfg = _STAGES_TUNED.get(key)
        if cfg is None:
            cfg = (0, 0, -1) if torch.cuda.is_current_stream_capturing() else _tune_conv(
                A, B, out, stats, bias, geo, dh, dw, tb, zero, addend, bwd, groups, scales, xa, xf, mask)
            if cfg[0] or cfg[2] >= 0:
                _STAGES_TUNED[key] = cfg
    if cfg[2] >= DEEP_BASE:
        DEEP_COUNT[0] += 1
    elif cfg[2] >= HALO_BASE:
        HALO_COUNT[0] += 1
    elif cfg[2] >= DIRECT_BASE:
        _direct_launch(A, B, out, stats, groups, _direct_geom(geo, dh, dw, tb, out, bias, addend, bwd, scales),
                       cfg[2] - DIRECT_BASE, bwd, shift)
        return
    C.conv_gemm(A, B, out, stats, bias, *geo, dh, dw, tb, groups, zero, addend, *bwd, *cfg, *scales, *xa3, shift,
                *xf2, mask, None, None, None, 0)


_CFGS = None


def conv_cfgs():
    """The bf16 kernel configuration table: (tile rows, tile channels, waves M, waves N, ring depth)."""
    global _CFGS
    if _CFGS is None:
        _CFGS = [tuple(c) for c in C.conv_cfgs()]
    return _CFGS


_HALO_CFGS = None
HALO_CONV = os.environ.get("IMGCLS_HALO", "1") == "1"  # halo-patch 3x3 kernels as tuner candidates
# entries the tuner times: only the 256 x 256 tile beat the LDS-DMA implicit GEMM on a ResNet-50 b1024 shape
# (512-channel 7x7: 266 vs 279 us); the others lost 1.3-2x (profiles/r6b_halo_probe_b1024.txt)
HALO_TUNE = tuple(int(v) for v in os.environ.get("IMGCLS_HALO_TUNE", "6").split(",") if v)
HALO_FORCE = None  # tests: force a halo variant on every eligible launch
HALO_COUNT = [0]   # halo-kernel launches (tests)
HALO_BASE = 1000   # cfg[2] >= HALO_BASE: the halo-patch kernel (csrc/conv_halo.hip), entry cfg - base


def conv_halo_cfgs():
    """The halo-patch kernel's table: (tile rows, tile channels, waves M, waves N, weight ring, patch rows)."""
    global _HALO_CFGS
    if _HALO_CFGS is None:
        _HALO_CFGS = [tuple(c) for c in C.conv_halo_cfgs()]
    return _HALO_CFGS


def _halo_ok(geo, dh, dw, tm, pmax):
    """The launch is a stride-1 GEMM whose taps lie in a 3x3 window over an input grid of the output's size
    (3x3 same-padded forward convs, stride-1 data gradients) and the tile's patch fits ``pmax`` rows - the
    same test as csrc/conv_halo.hip::halo_geometry."""
    m, _co, k, ca, gh, gw, ih, iw, sa = geo[:9]
    if ca % 64 or sa != 1 or gh != ih or gw != iw or not 2 <= len(dh) <= 9 or k != len(dh) * ca:
        return False
    if m % (ih * iw) or any(abs(v) > 1 for v in dh) or any(abs(v) > 1 for v in dw):
        return False
    return tm + 2 * iw + 2 <= pmax and pmax * ca * 2 < (1 << 30)


_DEEP_CFGS = None
DEEP_CONV = os.environ.get("IMGCLS_DEEP", "1") == "1"  # prefetch-depth-2 kernels (csrc/conv_deep.hip) as tuner candidates
DEEP_FORCE = None  # tests: force a deep variant on every eligible launch
DEEP_COUNT = [0]   # deep-kernel launches (tests)
DEEP_BASE = 2000   # cfg[2] >= DEEP_BASE: the prefetch-depth-2 kernel, entry cfg - base


def conv_deep_cfgs():
    """The prefetch-depth-2 kernel's table: (tile rows, tile channels, waves M, waves N, schedule variant);
    variants with bit 2 or 4 set are diagnostics (wrong results) the tuner never times."""
    global _DEEP_CFGS
    if _DEEP_CFGS is None:
        _DEEP_CFGS = [tuple(c) for c in C.conv_deep_cfgs()]
    return _DEEP_CFGS


def _deep_ok(geo, dh, dw):
    """Uniform 64-channel k-steps and 16-bit input coordinates (csrc/conv_deep.hip::conv_deep_launch)."""
    if geo[3] % 64:
        return False
    return (geo[6] <= 16383 and geo[7] <= 16383) or not any(dh) and not any(dw)


_FP8_CFGS = None


def conv_fp8_cfgs():
    """The MX-FP8 forward kernel's configuration table (same fields as ``conv_cfgs``)."""
    global _FP8_CFGS
    if _FP8_CFGS is None:
        _FP8_CFGS = [tuple(c) for c in C.conv_fp8_cfgs()]
    return _FP8_CFGS


def _conv_candidates(m, ncols, fp8, xa=False):
    """(stages, tile_n, cfg) triples worth timing for an M x Ncols GEMM (``xa``: configurations with
    fused BN-backward / BN-apply A-operand variants only)."""
    out = []
    for i, (tm, bn, _wm, _wn, _st) in enumerate(conv_fp8_cfgs() if fp8 else conv_cfgs()):
        if xa and not C.conv_cfg_has_xa(i):
            continue
        if bn > 64 and bn >= 2 * ncols:   # tile at least half empty
            continue
        if bn == 64 and ncols >= 512:     # 8+ column tiles re-read the pixel panel too often
            continue
        if bn == 32 and (ncols % 64 == 0 or ncols > 96):  # 32-wide tiles only where 64 would waste columns
            continue
        if tm == 256 and m < 256 * 16:    # too few row tiles to fill the chip
            continue
        out.append((0, 0, i))
    return out


DIRECT_CONV = os.environ.get("IMGCLS_DIRECT_CONV", "1") == "1"
DIRECT_FORCE = None  # tests: force a direct-kernel variant on every eligible launch
DIRECT_DGRAD = os.environ.get("IMGCLS_DIRECT_DGRAD", "1") == "1"  # data gradients (+ BN-backward epilogue)
DIRECT_BASE = 100  # cfg[2] >= DIRECT_BASE: the halo-tile direct kernel (csrc/direct_conv.hip), variant cfg - base
# variant -> (padded input channels, output-channel tile)
DIRECT_CFGS = {0: (32, 32), 1: (32, 64), 2: (64, 32), 3: (64, 64), 4: (96, 32)}


def _direct_geom(geo, dh, dw, tb, out, bias, addend, bwd, scales):
    """(N, H, W, Cin, OH, OW, Cout, pt, pl, tap order) when this launch is a stride-1 3x3 conv the direct
    kernel handles - a forward conv, or the single-phase data gradient of a stride-1 3x3 conv (a 3x3 conv
    of dY with the transposed, flipped weights), optionally with the fused BN-backward epilogue - with
    <= 96 input channels, a dense output and no addend / residual; else None.  The tap order maps the
    kernel's (th, tw) to the GEMM's weight tap (identity for the forward conv)."""
    m, co, k, cx, gh, gw, ih, iw, sa = geo[:9]
    if not DIRECT_CONV or scales[0] is not None or bias is not None or addend is not None or bwd[1] is not None:
        return None
    if bwd[0] is not None and not DIRECT_DGRAD:
        return None
    if sa != 1 or geo[12] != 1 or geo[13] or geo[14] or geo[15] != co or geo[16] or len(dh) != 9:
        return None
    if cx % 8 or cx > 96 or co % 8 or k != 9 * cx or m % (gh * gw) or out.shape[1] != co:
        return None
    pt, pl = -min(dh), -min(dw)
    order = [None] * 9
    for t in range(9):
        th, tw = dh[t] + pt, dw[t] + pl
        if not (0 <= th < 3 and 0 <= tw < 3) or order[th * 3 + tw] is not None:
            return None
        order[th * 3 + tw] = tb[t]
    if pt > 2 or pl > 2:
        return None
    return (m // (gh * gw), ih, iw, cx, gh, gw, co, pt, pl, tuple(order))


_ORDER_IDX: dict = {}


def _direct_launch(A, B, out, stats, groups, dg, variant, bwd, shift=None):
    n, ih, iw, cx, gh, gw, co, pt, pl, order = dg
    if order == tuple(range(9)):
        w = B
    else:  # tap permutation of the transposed weight; a cached device index (a host list would sync)
        key = (order, B.device)
        idx = _ORDER_IDX.get(key)
        if idx is None:
            idx = _ORDER_IDX[key] = torch.tensor(order, dtype=torch.long, device=B.device)
        w = B.view(co, 9, cx).index_select(1, idx)
    if bwd[0] is not None:  # fused BN-backward epilogue (BwdLink): partial rows instead of statistics
        C.direct_conv(A, w, out, bwd[3], bwd[5], n, ih, iw, cx, gh, gw, co, pt, pl, variant,
                      y_bn=bwd[0], coef=bwd[2], act=bwd[4])
    else:
        C.direct_conv(A, w, out, stats, groups, n, ih, iw, cx, gh, gw, co, pt, pl, variant, shift=shift)


def _tune_conv(A, B, out, stats, bias, geo, dh, dw, tb, zero, addend, bwd, groups, scales=(None, None), xa=None,
               xf=None, mask=None):
    scratch = torch.empty_like(out)
    sst = torch.zeros_like(stats) if stats is not None else None
    bwd = tuple(bwd)
    if bwd[3] is not None:
        bwd = bwd[:3] + (torch.zeros_like(bwd[3]),) + bwd[4:]
    fused = xa is not None or xf is not None
    cands = _conv_candidates(geo[0], geo[1], scales[0] is not None, fused)
    xa3 = (xa[0], xa[1], None) if xa is not None else (None, None, None)
    xf2 = (xf[0], xf[1]) if xf is not None else (None, 0)
    times = {}
    for cfg in cands:
        times[cfg] = _time_ms(lambda: C.conv_gemm(A, B, scratch, sst, bias, *geo, dh, dw, tb, groups, zero,
                                                  addend, *bwd, *cfg, *scales, *xa3, None, *xf2, mask, None, None, None, 0))
    if HALO_CONV and not fused and scales[0] is None:
        for v, (tm, bn, _wm, _wn, _bst, pmax) in enumerate(conv_halo_cfgs()):
            if v not in HALO_TUNE or not _halo_ok(geo, dh, dw, tm, pmax) or (bn > 64 and bn >= 2 * geo[1]) or \
                    (bn == 64 and geo[1] >= 256) or geo[0] < tm * 16:
                continue
            cfg = (0, 0, HALO_BASE + v)
            times[cfg] = _time_ms(lambda: C.conv_gemm(A, B, scratch, sst, bias, *geo, dh, dw, tb, groups, zero,
                                                      addend, *bwd, *cfg, *scales, *xa3, None, *xf2, mask, None, None, None, 0))
    if DEEP_CONV and not fused and scales[0] is None and _deep_ok(geo, dh, dw):
        for v, (tm, bn, _wm, _wn, var) in enumerate(conv_deep_cfgs()):
            if var & 6 or (bn > 64 and bn >= 2 * geo[1]) or (bn == 64 and geo[1] >= 256) or geo[0] < tm * 8:
                continue
            cfg = (0, 0, DEEP_BASE + v)
            times[cfg] = _time_ms(lambda: C.conv_gemm(A, B, scratch, sst, bias, *geo, dh, dw, tb, groups, zero,
                                                      addend, *bwd, *cfg, *scales, *xa3, None, *xf2, mask, None, None, None, 0))
    dg = _direct_geom(geo, dh, dw, tb, out, bias, addend, bwd, scales) if not fused else None
    if dg is not None:
        for v, (cip, cot) in DIRECT_CFGS.items():
            if dg[3] <= cip and (cot == 32 or dg[6] > 32):
                times[(0, 0, DIRECT_BASE + v)] = _time_ms(
                    lambda: _direct_launch(A, B, scratch, sst, groups, dg, v, bwd))
    TUNE_LOG.append((geo[0], geo[1], geo[2], times))
    return min(times, key=times.get)


def fp8_eligible(g: "ConvGeom") -> bool:
    return FP8_FWD and g.Cx == g.Ci and g.Cx % 128 == 0 and g.Co % 8 == 0


def conv_forward_raw(x, w_param, g: ConvGeom, stats=None, bias=None, out=None, c_off=0, wb=None, shift=None,
                     xf=None):
    """``xf`` = (coef, act): x holds a BN's input y; the conv reads act(bn(y)) (``XfHold``)."""
    dev = x.device
    if wb is None and xf is None and fp8_eligible(g):
        return _conv_forward_fp8(x, w_param, g, stats, bias, out, c_off, shift)
    if wb is None:
        wb = _weight_for_input(w_param, g.Cx)
    y = out if out is not None else _empty_cl(g.N, g.Co, g.OH, g.OW, dev)
    ldc = y.shape[1]
    dh, dw, tb = _fwd_taps(g)
    if g.sh != g.sw:
        raise NotImplementedError("anisotropic stride")
    geo = (g.N * g.OH * g.OW, g.Co, g.T * g.Cx, g.Cx, g.OH, g.OW, g.H, g.W, g.sh, g.T * g.Cx, g.OH, g.OW,
           1, 0, 0, ldc, c_off)
    _conv_gemm(x, wb, y, stats, bias, geo, dh, dw, tb, ws(dev).zero, groups=stat_groups(geo[0]), shift=shift,
               xf=xf)
    return y


def _conv_forward_fp8(x, w_param, g: ConvGeom, stats, bias, out, c_off, shift=None):
    dev = x.device
    xq, xs = act_mx(x)
    wq, wsc = weight_mx(w_param)
    y = out if out is not None else _empty_cl(g.N, g.Co, g.OH, g.OW, dev)
    dh, dw, tb = _fwd_taps(g)
    geo = (g.N * g.OH * g.OW, g.Co, g.T * g.Cx, g.Cx, g.OH, g.OW, g.H, g.W, g.sh, g.T * g.Cx, g.OH, g.OW,
           1, 0, 0, y.shape[1], c_off)
    _conv_gemm(xq, wq, y, stats, bias, geo, dh, dw, tb, ws(dev).zero, groups=stat_groups(geo[0]),
               scales=(xs, wsc), shift=shift)
    return y


# Fused XA backward of a 1x1 stride-1 conv with 64 input channels (ResNet layer1 conv3, csrc/conv_gemm.hip
# conv_fused_bwd_kernel): one pass over dz and y feeds both the data gradient (+ its BN-backward epilogue) and
# the weight gradient, instead of each GEMM reading dz and y (IMGCLS_FUSED_BWD=0: separate launches).
FUSED_XA_BWD = os.environ.get("IMGCLS_FUSED_BWD", "1") == "1"
FUSED_XA_BWD_COUNT = [0]  # fused dgrad + wgrad launches (tests / diagnostics)
# the 64-output form (layer1 conv1: dgrad columns walked in 64-channel chunks) measured slower than the separate
# launches (ResNet-50 b1024 13344-13358 vs 13589-13626 img/s with only the 64-input form, profiles/r7n_*): off
FUSED_XA_BWD_N = os.environ.get("IMGCLS_FUSED_BWD_N", "0") == "1"
_CU_COUNT: dict = {}


def fused_bwd_eligible(g: ConvGeom, xa) -> bool:
    if not (FUSED_XA_BWD and xa is not None and g.kh == 1 and g.kw == 1 and g.sh == 1 and g.sw == 1
            and g.pt == 0 and g.pl == 0 and g.Cx == g.Ci and g.OH == g.H and g.OW == g.W):
        return False
    # 64 input channels and up to 256 outputs (layer1 conv3), or 64 outputs and 128 / 256 inputs (layer1 conv1)
    return (g.Ci == 64 and g.Co % 64 == 0 and g.Co <= 256) or (FUSED_XA_BWD_N and g.Co == 64 and g.Ci in (128, 256))


def conv_fused_bwd_raw(dz, x, w_param, g: ConvGeom, xa, addend=None, link=None):
    """dX (as ``conv_dgrad_raw`` with ``xa``) and dW (into the parameter's arena slot or a fresh gradient
    buffer) of a ``fused_bwd_eligible`` conv from one launch; returns (dx, dw)."""
    dev = dz.device
    bwd = (None, None, None, None, 0, 1)
    mask = None
    if link is not None:
        grp = stat_groups(g.N * g.H * g.W)
        link.part = ws(dev).take_part(g.Ci, grp)
        bwd = (link.y, link.res, link.coef, link.part, link.act, grp)
        mask = link.mask
    wt = weight_bf16_t(w_param, g.Co, g.T, g.Ci)
    dx = _empty_cl(g.N, g.Ci, g.H, g.W, dev)
    dw = arena_slot(w_param)
    if dw is None:
        dw = grad_buffer(w_param)
    blocks = _CU_COUNT.get(dev.index)
    if blocks is None:
        blocks = _CU_COUNT[dev.index] = torch.cuda.get_device_properties(dev).multi_processor_count
    wsp = _wgrad_ws(dev, blocks * g.Co * g.Ci)
    m = g.N * g.H * g.W
    geo = (m, g.Ci, g.Co, g.Co, g.H, g.W, g.OH, g.OW, 1, g.Co, g.H, g.W, 1, 0, 0, g.Ci, 0)
    C.conv_gemm(dz, wt, dx, None, None, *geo, [0], [0], [0], G_STATS, ws(dev).zero, addend, *bwd, 0, 0, -1, None, None,
                xa[0], xa[1], None, None, None, 0, mask, x, wsp, dw.view(-1), blocks)
    FUSED_XA_BWD_COUNT[0] += 1
    return dx, dw


def conv_dgrad_raw(dy, w_param, g: ConvGeom, addend=None, link=None, xa=None):
    """dX = conv_transpose(dY, W) [+ addend], one MFMA GEMM per sub-pixel phase.

    With ``link`` (the producer BN of the conv input) the epilogue instead emits
    dz = act'(z) * dX and the producer's BN-backward partial sums (fused reduce).
    With ``xa`` = (y, coef) ``dy`` is the consuming BN's pre-elementwise gradient dz and the kernel
    forms dY = coef0*dz + coef1*y + coef2 on its A-operand loads (1x1 convs, ``XaLink``)."""
    dev = dy.device
    bwd = (None, None, None, None, 0, 1)
    mask = None
    if link is not None:
        grp = stat_groups(g.N * g.H * g.W)
        link.part = ws(dev).take_part(g.Ci, grp)
        bwd = (link.y, link.res, link.coef, link.part, link.act, grp)
        mask = link.mask
    wt = weight_bf16_t(w_param, g.Co, g.T, g.Ci)
    dx = _empty_cl(g.N, g.Ci, g.H, g.W, dev)
    for ph, pw, gh, gw, dh, dw, tb in _dgrad_phases(g):
        if gh <= 0 or gw <= 0:
            continue
        geo = (g.N * gh * gw, g.Ci, len(tb) * g.Co, g.Co, gh, gw, g.OH, g.OW, 1, g.T * g.Co, g.H, g.W, g.sh,
               ph, pw, g.Ci, 0)
        _conv_gemm(dy, wt, dx, None, None, geo, dh, dw, tb, ws(dev).zero, addend, bwd,
                   xa=xa if len(tb) else None, mask=mask)
    return dx


WGRAD_TARGET_BLOCKS = int(os.environ.get("IMGCLS_WGRAD_BLOCKS", "0"))  # 0 = autotune per shape
WGRAD_TUNE_LOG: list = []  # (Co, Ntot, pixels, {(blocks, stages): ms}) per tuned wgrad shape
WGRAD_MIN_K = int(os.environ.get("IMGCLS_WGRAD_MIN_K", "512"))
WGRAD_CANDIDATES = tuple(int(v) for v in os.environ.get("IMGCLS_WGRAD_CANDS", "256,384,512,768,1024,1536,2048").split(","))
_WGRAD_TUNED: dict = {}


def _wgrad_split(m, tiles, target):
    splits = max(1, min(-(-target // max(tiles, 1)), -(-m // WGRAD_MIN_K)))
    kps = -(-m // splits)
    kps = -(-kps // 64) * 64
    splits = -(-m // kps)
    return kps, splits


WGRAD_NARROW_TILES = os.environ.get("IMGCLS_WGRAD_NARROW_TILES", "1") == "1"  # stages 10-12 as tuner candidates
WGRAD_STAGES = int(os.environ.get("IMGCLS_WGRAD_STAGES", "0"))  # 0 = tuned with the split count; 1 | 2 | 3


WGRAD_WS = os.environ.get("IMGCLS_WGRAD_WS", "1") == "1"  # split-K partials: workspace slabs + reduce (0: atomics)
_WGRAD_WS: dict = {}  # (device index, stream id) -> fp32 workspace, grown on demand


def _wgrad_ws(dev, n):
    """Split-K workspace of at least ``n`` floats for launches on the current stream (one per stream:
    launches on one stream run in order, so consecutive layers share it)."""
    key = (dev.index, torch.cuda.current_stream(dev).stream_id)
    buf = _WGRAD_WS.get(key)
    if buf is None or buf.numel() < n:
        buf = _WGRAD_WS[key] = torch.empty(max(n, 1 << 20), dtype=torch.float32, device=dev)
    return buf


# diagnostic only (scripts/gpu_*.sh contention studies; never a benchmark number): skip the weight-gradient
# GEMMs to time the compute stream without the side stream's load.  bench.py refuses to report with it set.
SKIP_WGRAD = os.environ.get("IMGCLS_DIAG_SKIP_WGRAD", "0") == "1"


def _wgrad_launch(dy, x, out, g: ConvGeom, m, ntot, kps, splits, stages=2, side=None, xa=None, xf=None):
    """One weight-gradient launch on the current stream, or (``side``: a ``_SideStream``) forked onto the
    side stream inside the launcher (event record / wait and allocator stream records in C++).  ``xa`` =
    (y, coef): dy is a BN's pre-elementwise gradient, the kernel applies the elementwise map itself.
    ``xf`` = (coef, act): x is a BN's input y, the kernel reads act(bn(y))."""
    if SKIP_WGRAD:
        return
    wsp = None
    if WGRAD_WS and splits > 1 and ntot % 8 == 0:
        n = splits * g.Co * ntot
        if side is None:
            wsp = _wgrad_ws(dy.device, n)
        else:
            if side.ws is None or side.ws.numel() < n:
                side.ws = torch.empty(max(n, 1 << 20), dtype=torch.float32, device=dy.device)
            wsp = side.ws
    C.conv_wgrad(dy, x, out, m, g.Co, g.Cx, ntot, g.OH, g.OW, g.H, g.W, g.sh, g.sw, g.pt, g.pl,
                 g.dil, g.dil, g.kw, kps, splits, ws(dy.device).zero, stages, wsp, side.handle if side else 0,
                 xa_y=xa[0] if xa is not None else None, xa_coef=xa[1] if xa is not None else None,
                 xf_coef=xf[0] if xf is not None else None, xf_act=xf[1] if xf is not None else 0)


def _wgrad_tiles(co, ntot, stages):
    """Output tiles of one wgrad launch: 256 x 256 for the 8-wave kernels (stages 4, 7, 9), 32 x 128 for
    stages 5 / 6, 64-column tiles for stages 10 / 11 (64|128 rows) and 12 (256 rows), else 64|128 x 128."""
    if stages in (4, 7, 9):
        return (-(-co // 256)) * (-(-ntot // 256))
    if stages >= 10:
        return (-(-co // (256 if stages == 12 else 64 if co <= 64 else 128))) * (-(-ntot // 64))
    return (-(-co // (32 if stages in (5, 6) else 64 if co <= 64 else 128))) * (-(-ntot // 128))


def _wgrad_plan(g: ConvGeom, dy, x, m, ntot, xa=None, xf=None):
    """(k_per_split, splits, stages) of the weight-gradient launch for this geometry."""
    target, stages = _wgrad_config(dy, x, g, m, ntot, xa, xf)
    kps, splits = _wgrad_split(m, _wgrad_tiles(g.Co, ntot, stages), target)
    return kps, splits, stages


def _wgrad_has(st, fx, ff):
    return (not fx or C.conv_wgrad_has_xa(st)) and (not ff or C.conv_wgrad_has_xf(st))


def _wgrad_config(dy, x, g: ConvGeom, m, ntot, xa=None, xf=None):
    """(split-K block target, LDS ring depth): fixed by IMGCLS_WGRAD_BLOCKS / IMGCLS_WGRAD_STAGES,
    else timed jointly once per shape (cached).  With ``xa`` (fused BN-backward dY) only the variants
    that have the fused form are candidates, and they are timed with it.

    Tuning runs on a scratch gradient buffer, outside any graph capture, the first time a shape
    is seen (warmup), like a conv-algorithm "find" step."""
    fx, ff = xa is not None, xf is not None
    if DETERMINISTIC:  # one split: every dW element receives exactly one atomic contribution
        return 1, (WGRAD_STAGES if WGRAD_STAGES and _wgrad_has(WGRAD_STAGES, fx, ff) else 2)
    blocks = (WGRAD_TARGET_BLOCKS,) if WGRAD_TARGET_BLOCKS > 0 else WGRAD_CANDIDATES
    stages = (WGRAD_STAGES,) if WGRAD_STAGES > 0 and _wgrad_has(WGRAD_STAGES, fx, ff) else (1, 2)
    if len(blocks) == 1 and len(stages) == 1:
        return blocks[0], stages[0]
    key = ((g.N, g.Cx, g.H, g.W, g.Co, g.kh, g.kw, g.sh, g.pt, g.pl, g.dil, blocks, stages) + ((True,) if fx else ())
           + (("xf",) if ff else ()))
    best = _WGRAD_TUNED.get(key)
    if best is not None:
        return best
    if torch.cuda.is_current_stream_capturing():
        return blocks[len(blocks) // 2], stages[-1]
    scratch = torch.zeros(g.Co * ntot, dtype=torch.float32, device=dy.device)
    times = {}
    cands = [(cand, st) for st in stages for cand in blocks]
    if WGRAD_STAGES == 0:
        # 8-wave blocks (in-block 2-way pixel split, one block per CU): fewer, larger blocks
        cands += [(cand, 3) for cand in blocks if cand <= 1024]
        if g.Co >= 256 and ntot >= 256:  # 256 x 256 tiles on 8 waves, ~1-2 blocks per CU
            cands += [(cand, st) for st in (4, 7, 9) for cand in (256, 512)]
        # 4-deep ring of 32-pixel stages (two stages in flight across every barrier), 4 waves
        cands += [(cand, 8) for cand in blocks if cand <= 1024]
        if g.Co <= 32:  # 32-row tiles: a 64-row tile would be half empty
            cands += [(cand, st) for st in (5, 6) for cand in blocks]
        if ntot <= 64 and WGRAD_NARROW_TILES:  # 64-column tiles: a 128-column tile is half empty (layer1 conv3)
            cands += [(cand, st) for st in (10, 11) for cand in blocks]
            if g.Co >= 256:
                cands += [(cand, 12) for cand in blocks if cand <= 1024]
        # (64 / 128 x 256 four-wave tiles, reading the narrow layers' dY half as often, were 5-70 % slower
        # on every ResNet-50 shape: profiles/r4d_wgrad_wide_tiles_probe.txt)
    if fx or ff:
        cands = [(cand, st) for cand, st in cands if _wgrad_has(st, fx, ff)]
    for cand, st in cands:
        kps, splits = _wgrad_split(m, _wgrad_tiles(g.Co, ntot, st), cand)
        times[(cand, st)] = _time_ms(lambda: _wgrad_launch(dy, x, scratch, g, m, ntot, kps, splits, st, xa=xa,
                                                           xf=xf))
    best = min(times, key=times.get)
    _WGRAD_TUNED[key] = best
    WGRAD_TUNE_LOG.append((g.Co, ntot, m, times))
    return best


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
# (Inception-v3 b128: 3303 vs 6523 img/s, profiles/r3g_hip_graph_modes.txt); IMGCLS_GRAPH_SIDE=1 forks
GRAPH_SIDE = os.environ.get("IMGCLS_GRAPH_SIDE", "0") == "1"
_SIDE: dict = {}  # device index -> _SideStream


class _SideStream:
    __slots__ = ("stream", "joins", "handle", "ws")

    def __init__(self, dev):
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
    from ..parallel import comm_timer
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
                _wgrad_launch(dy, x, dw, g, m, ntot, kps, splits, stages, xa=xa, xf=xf)
                return dw
            if not s.joins:  # first side launch of this backward: join when the engine finishes
                torch.autograd.Variable._execution_engine.queue_callback(join_side_streams)
            s.joins.add(torch.cuda.current_stream(dev))
            _wgrad_launch(dy, x, dw, g, m, ntot, kps, splits, stages, side=s, xa=xa, xf=xf)
            return dw
        dw = grad_buffer(w_param)
        _wgrad_launch(dy, x, dw, g, m, ntot, kps, splits, stages, xa=xa, xf=xf)
        return dw
    full = torch.zeros(g.Co * ntot, dtype=torch.float32, device=dev)
    dw = arena_slot(w_param)
    if dw is not None:
        # padded input channels = the network's input layer, the last weight gradient of backward: on the
        # compute stream (idle by then) it runs beside the side stream's backlog instead of behind it - the
        # ResNet-50 b1024 stem wgrad is ~0.7 ms of the step tail (profiles/r5e_conv_roofline_b1024.txt)
        if STEM_WGRAD_SIDE:
            def launch():
                _wgrad_launch(dy, x, full, g, m, ntot, kps, splits, stages)
                C.grad_unpad(full, dw, g.Co * g.T, g.Cx, g.Ci)
            _on_side(dev, launch, dy, x, full)
            return dw
        _wgrad_launch(dy, x, full, g, m, ntot, kps, splits, stages)
        C.grad_unpad(full, dw, g.Co * g.T, g.Cx, g.Ci)
        return dw
    _wgrad_launch(dy, x, full, g, m, ntot, kps, splits, stages)
    dw = grad_buffer(w_param, zero=False)
    C.grad_unpad(full, dw, g.Co * g.T, g.Cx, g.Ci)
    return dw


class GradSlot:
    """Collects the backward contributions of the ``n`` consumers of one tensor (a ResNet block input
    feeding conv1 and the identity / downsample branch: n=2; an Inception block input feeding three
    convs and a pool: n=4).  Each consumer to run backward adds the running sum - inside its dgrad
    epilogue when it is a convolution - and parks the result, reporting no gradient to autograd; the
    consumer that completes the sum hands it over.  Autograd's separate accumulation passes disappear.
    Order-independent; every one of the ``n`` consumers must deliver exactly once."""

    __slots__ = ("t", "n", "seen")

    def __init__(self, n: int = 2):
        self.t = None
        self.n = n
        self.seen = 0

    def completes(self) -> bool:
        """True when the next delivery is the last one (the producer's full gradient)."""
        return self.seen == self.n - 1

    def deliver(self, grad, fused=False):
        """Return what the consumer should hand to autograd.  ``fused``: ``grad`` already includes
        the parked running sum (it was the consumer's dgrad addend)."""
        self.seen += 1
        if not fused and self.t is not None:
            out = torch.empty_like(grad, memory_format=CL)
            C.add(_cl(grad), _cl(self.t), out)
            grad = out
        if self.seen < self.n:
            self.t = grad
            return None
        self.t = None
        return grad


PEER_BN_MAX_C = int(getattr(C, "PEER_BN_MAX_C", 0))  # channels the fused SyncBN peer kernels handle
C.bn_set_unroll(os.environ.get("IMGCLS_BN_UNROLL", "1") == "1")  # U-row BN elementwise kernels
SYNCBN_EARLY_COUNT = [0]  # SyncBN backward all-reduces launched from the consuming conv (tests)


def _syncbn_bwd_start(link):
    """Reduce the fused partial rows to this rank's [sum dz, sum dz*xhat] (+ dgamma, dbeta) and launch
    the async cross-rank all-reduce; ``BNActFn.backward`` waits on it (a stream wait, no host sync).
    With the peer transport one side-stream kernel does the reduce, the exchange and k = sums / n."""
    c = link.c
    dev = link.y.device
    dgamma = grad_buffer(link.params[0], zero=False)
    dbeta = grad_buffer(link.params[1], zero=False)
    pc = peer_channel(link.group, 1)
    if pc is not None and link.count_t is not None and c <= PEER_BN_MAX_C:
        k = torch.empty(2 * c, dtype=torch.float32, device=dev)
        cur = torch.cuda.current_stream(dev)
        side = peer_side_stream(dev)
        side.wait_stream(cur)
        from ..parallel import comm_timer
        with torch.cuda.stream(side):
            with comm_timer.span("syncbn_bwd", side):
                pc.comm.bn_bwd(link.part, link.part_rows(), c, link.count_t, dgamma, dbeta, k)
            ev = torch.cuda.Event()
            ev.record(side)
        for t in (k, link.count_t, dgamma, dbeta):
            t.record_stream(side)
        link.pending = (None, PeerWork(ev), dgamma, dbeta, k)
    else:
        sums = torch.empty(2 * c, dtype=torch.float64, device=dev)
        C.bn_partials(link.part, link.part_rows(), c, sums, dgamma, dbeta)
        work = stats_all_reduce_async(sums, link.group)
        link.pending = (sums, work, dgamma, dbeta, None)
    SYNCBN_EARLY_COUNT[0] += 1


class BwdLink:
    """Ties a BN(+act) output to the conv that consumes it, so the consumer's dgrad epilogue can run
    the producer's BN-backward reduce (``done`` tells the producer its gradient arrives as dz)."""

    __slots__ = ("y", "coef", "res", "mask", "act", "part", "done", "group", "params", "pending", "c", "rows",
                 "groups", "count_t")

    def __init__(self):
        self.y = self.coef = self.res = self.mask = self.part = None
        self.act = 0
        self.done = False
        self.group = self.params = self.pending = None  # SyncBN: early backward all-reduce
        self.c = self.rows = 0
        self.groups = 0  # partial rows in ``part`` (0: stat_groups(rows), the GEMM epilogue's rotating rows)
        self.count_t = None  # SyncBN: all-reduced element count of the forward (fp64 device scalar)

    def part_rows(self) -> int:
        return self.groups or stat_groups(self.rows)


# BN-backward elementwise fused into the producer conv's gradient GEMMs (csrc/conv_gemm.hip XA):
# for a 1x1 conv followed by BN, the BN backward hands the conv its pre-elementwise gradient dz and the
# per-channel affine map dY = c0*dz + c1*y + c2 instead of writing dY with bn_bwd_elemt; the conv's dgrad
# and wgrad kernels form dY on their operand loads.  (Before: elemt read dz and y and wrote dY, then both
# GEMMs read dY - the BN elementwise passes were 37 % of the ResNet-50 step)
FUSE_XA = os.environ.get("IMGCLS_BN_XA", "1") == "1"
XA_COUNT = [0]  # BN backwards handed to their producer conv (tests / diagnostics)
# A fused operand map is applied every time the GEMM loads the element: once per tap that gathers it and
# once per tile along the GEMM's other dimension.  The unfused pass touches each element once (memory-
# bound), so fusing pays only while that replication stays small (docs/DESIGN.md, "what fusion costs").
XA_MAX_REP = int(os.environ.get("IMGCLS_XA_MAX_REP", "2"))
XA_NARROW_OFF = os.environ.get("IMGCLS_XA_NARROW_OFF", "0") == "1"
XF_MAX_REP = int(os.environ.get("IMGCLS_XF_MAX_REP", "2"))


def _rep(taps: int, other: int) -> int:
    """Times a fused operand map runs per element: taps x tiles of (up to) 256 along the other dimension."""
    return taps * max(1, -(-other // 256))


class XaLink:
    """Ties a 1x1 conv to the BN consuming its output y for the fused backward: the BN's backward parks
    (dz, y, coef [3][C]) here and returns dz as the conv output's gradient; the conv's backward checks
    that it received exactly that tensor and runs its dgrad / wgrad with the fused operand map."""

    __slots__ = ("dz", "y", "coef")

    def __init__(self):
        self.dz = self.y = self.coef = None

    def take(self, dy):
        """(y, coef) when ``dy`` is the parked dz (and clears the link), else None."""
        if self.dz is None:
            return None
        if dy.data_ptr() != self.dz.data_ptr() or dy.shape != self.dz.shape:
            raise RuntimeError("fused BN backward: the conv received a gradient other than its BN's dz")
        out = (self.y, self.coef)
        self.dz = self.y = self.coef = None
        return out


def xa_eligible(x, conv) -> bool:
    """A dense conv (no bias / groups / dilation, square stride) whose output channels are a multiple of 64
    (uniform k-steps of the dgrad GEMM, K = taps x Cout) and whose input channels are unpadded: its backward
    can take the fused BN-backward operand map (padded taps are masked in the kernel)."""
    taps = conv.kernel_size[0] * conv.kernel_size[1]
    if XA_NARROW_OFF and conv.out_channels <= 64 and conv.in_channels > 64:
        return False  # (diagnostic knob) the narrow-output XA weight gradient
    return (FUSE_XA and conv.stride[0] == conv.stride[1] and tuple(conv.dilation) == (1, 1)
            and conv.groups == 1 and conv.bias is None and conv.out_channels % 64 == 0
            and x.shape[1] == conv.in_channels and conv.in_channels % 8 == 0 and taps <= 49
            # dgrad: dz gathered by every tap, per tile of the input channels; wgrad: per column tile
            and max(_rep(taps, conv.in_channels), _rep(1, taps * conv.in_channels)) <= XA_MAX_REP)


# BN apply (+ReLU) fused into the consuming conv (csrc/conv_gemm.hip XF): a BN whose output only
# feeds one conv hands that conv its input y and its [scale | shift] instead of writing act(bn(y)); the
# conv's forward and weight-gradient kernels form act(scale * y + shift) on their operand loads, padded taps
# kept at zero.  The activated tensor is never written or re-read (VERDICT round 2, item 1 "forward").
# Off by default: measured on ResNet-50 b1024 (profiles/r5f_fusion_ab.txt) it does not pay - the bn_apply passes
# it removes are small (the non-residual ones were 3.5 ms of the 77 ms step) and a 3x3 consumer re-applies the
# map once per tap
FUSE_XF = os.environ.get("IMGCLS_BN_XF", "0") == "1"
XF_COUNT = [0]  # convs that read a deferred BN output (tests / diagnostics)


class XfHold:
    """The deferred BN output's map: ``coef`` = the BN's [scale | shift | mean | invstd] (written by its
    forward), ``act`` = 0 (identity) or 1 (ReLU).  Rides on the BN's output tensor as ``_imgcls_xf``; that
    tensor holds y (the BN input), so only a conv taking the map (``ConvFn``) or ``XfMaterializeFn`` may
    read it."""

    __slots__ = ("coef", "act")

    def __init__(self):
        self.coef = None
        self.act = 0


def xf_eligible(x, conv) -> bool:
    """The conv can read a deferred BN output: dense (no bias / groups / dilation, square stride), input
    channels a multiple of 64 (uniform k-steps of the forward GEMM, K = taps x Cin), not a dense layer
    (``DenseConvFn``)."""
    taps = conv.kernel_size[0] * conv.kernel_size[1]
    return (conv.stride[0] == conv.stride[1] and tuple(conv.dilation) == (1, 1) and conv.groups == 1
            and conv.bias is None and x.shape[1] == conv.in_channels and conv.in_channels % 64 == 0
            and taps <= 49 and not getattr(conv, "tf_same", False)
            # forward and wgrad: y gathered by every tap, per tile of the output channels
            and _rep(taps, conv.out_channels) <= XF_MAX_REP
            and not FP8_FWD and not dense_conv_eligible(x, conv))


class XfMaterializeFn(torch.autograd.Function):
    """act(bn(y)) of a deferred BN output for a consumer that cannot take the map (one bn_apply pass -
    what the BN would have written).  The gradient passes through: it is the gradient w.r.t. act(bn(y)),
    which is what the deferred output stands for."""

    @staticmethod
    def forward(ctx, y, hold):
        n, c, h, w = y.shape
        out = _empty_cl(n, c, h, w, y.device)
        C.bn_apply(y, hold.coef, None, out, n * h * w, c, c, 0, hold.act)
        return out

    @staticmethod
    def backward(ctx, g):
        return g, None


def materialize_deferred(x):
    """x itself, or act(bn(y)) when x is a deferred BN output (``XfHold``)."""
    hold = getattr(x, "_imgcls_xf", None)
    return x if hold is None else XfMaterializeFn.apply(x, hold)


class ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, conv, want_stats, slot=None, fuse_bwd=False, xa=None, shift=None, xf=None):
        g = conv_geom(x, conv)
        stats = ws(x.device).stats_buf(g.Co, stat_groups(g.N * g.OH * g.OW)) if want_stats else None
        xfm = (xf.coef, xf.act) if xf is not None else None
        y = conv_forward_raw(x, w, g, stats=stats, shift=shift if want_stats else None, xf=xfm)
        if xf is not None:
            XF_COUNT[0] += 1
        ctx.g = g
        ctx.slot = slot
        ctx.xa = xa
        ctx.xf = xfm
        link = getattr(x, "_imgcls_link", None) if (fuse_bwd or slot is not None) else None
        ctx.link = link if (link is not None and link.y is not None and g.Cx == g.Ci) else None
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        g = ctx.g
        dy = _cl(dy)
        xa = ctx.xa.take(dy) if ctx.xa is not None else None
        dx = None
        if ctx.needs_input_grad[0]:
            slot, link = ctx.slot, ctx.link
            if link is not None and link.done:
                link = None
            if slot is not None and not slot.completes():
                link = None  # the producer's BN reduce needs the full gradient
            # running sum of the other consumers' contributions rides in as the dgrad addend
            addend = slot.t if (slot is not None and g.Cx == g.Ci) else None
            if ctx.needs_input_grad[1] and ctx.xf is None and fused_bwd_eligible(g, xa):  # (XF: X is y, not act(bn(y)))
                dx, dw_fused = conv_fused_bwd_raw(dy, x, w, g, xa, addend=addend, link=link)
            else:
                dw_fused = None
                dx = conv_dgrad_raw(dy, w, g, addend=addend, link=link, xa=xa)
            if link is not None:
                link.done = True
                if link.group is not None:
                    # SyncBN: start the producer BN's backward all-reduce now, so its latency overlaps
                    # this conv's weight gradient instead of sitting between two dependent kernels
                    _syncbn_bwd_start(link)
            if slot is not None:
                dx = slot.deliver(dx, fused=addend is not None)
        else:
            dw_fused = None
        if dw_fused is not None:
            dw = dw_fused
        else:
            dw = conv_wgrad_raw(dy, x, w, g, xa=xa, xf=ctx.xf) if ctx.needs_input_grad[1] else None
        return dx, dw, None, None, None, None, None, None, None


# ---------------------------------------------------------------------------
# space-to-depth stem: 7x7 stride-2 conv of a 3-channel image
# ---------------------------------------------------------------------------
# y = conv7x7/s2/p3(x) equals a stride-1 4x4 conv (pad 2 top/left, 1 bottom/right) over
# s2d(x)[n][i][j][(dy*2+dx)*3 + c] = x[n][c][2i+dy][2j+dx] (16 channels, 12 used) with
# W'[co][ta][tb][(dy*2+dx)*3 + c] = W[co][c][2ta+dy-1][2tb+dx-1] (0 outside the 7x7 window).
# K shrinks from 49 taps x 8 padded channels (392, 37 % useful) to 256 (57 % useful), and every
# 64-wide k-step of the implicit GEMM is 4 adjacent pixels x 16 channels = 128 contiguous bytes
# (the 8-channel form gathers 16-byte pieces).
STEM_S2D = os.environ.get("IMGCLS_STEM_S2D", "1") == "1"
STEM_DIRECT = os.environ.get("IMGCLS_STEM_DIRECT", "1") == "1"  # stem.hip instead of the implicit GEMM
_S2D_INDEX: dict = {}


def stem_s2d_conv(conv) -> bool:
    """The 7x7 stride-2 3-channel stem conv the space-to-depth form serves."""
    return (STEM_S2D and conv.groups == 1 and conv.bias is None and conv.in_channels == 3
            and tuple(conv.kernel_size) == (7, 7) and tuple(conv.stride) == (2, 2)
            and tuple(conv.padding) == (3, 3) and tuple(conv.dilation) == (1, 1)
            and not getattr(conv, "tf_same", False))


def stem_s2d_eligible(x, conv) -> bool:
    """fp32 NCHW images of even size (the stem converts them), or a batch the loader already converted to
    the space-to-depth layout (``input_from_u8``)."""
    if getattr(x, "_imgcls_s2d", None) is not None:
        return stem_s2d_conv(conv)
    return (x.dim() == 4 and x.shape[1] == 3 and x.dtype == torch.float32
            and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0 and stem_s2d_conv(conv))


def input_from_u8(u8, spec, mean, std):
    """uint8 NHWC RGB batch on the GPU -> the model's first-layer input in ONE kernel:
    ``(u / 255 - mean) / std`` (reference dp/loader.py:86-91) and the model's own per-channel affine
    (Inception transform_input) folded into ``u * a + b``, written as bf16 either in the 16-channel
    space-to-depth stem layout (``spec[0]``, ResNet) or NHWC padded to 8 channels.  Replaces
    normalize_u8 (fp32 NCHW) + prepare_input / prepare_input_s2d (a second pass over that fp32 tensor).
    The result carries a marker so prepare_input / the stem pass it through unchanged."""
    s2d, sc, sh = spec
    n, h, w, _ = u8.shape
    a = [1.0 / (255.0 * std[c]) for c in range(3)]
    b = [-mean[c] / std[c] for c in range(3)]
    if sc is not None:
        a = [a[c] * sc[c] for c in range(3)]
        b = [b[c] * sc[c] + sh[c] for c in range(3)]
    if s2d:
        y = _empty_cl(n, 16, h // 2, w // 2, u8.device)
        C.input_u8(u8, y, a, b, 1)
        y._imgcls_s2d = (h, w)
    else:
        y = _empty_cl(n, 8, h, w, u8.device)
        C.input_u8(u8, y, a, b, 0)
        y._imgcls_prepared = True
    return y


def _s2d_index(dev):
    """KRSC position r*21 + s*3 + c of the 7x7x3 weight -> position in the 4x4x16 s2d weight."""
    idx = _S2D_INDEX.get(dev)
    if idx is None:
        pos = []
        for r in range(7):
            for c_ in range(7):
                for ch in range(3):
                    ta, dy = divmod(r + 1, 2)
                    tb, dx = divmod(c_ + 1, 2)
                    pos.append(ta * 64 + tb * 16 + (dy * 2 + dx) * 3 + ch)
        idx = _S2D_INDEX[dev] = torch.tensor(pos, dtype=torch.long, device=dev)
    return idx


def _s2d_geom(n, h, w, co) -> ConvGeom:
    g = ConvGeom.__new__(ConvGeom)
    g.taps = g.phases = None
    g.N, g.Ci, g.Cx, g.H, g.W, g.Co = n, 16, 16, h // 2, w // 2, co
    g.kh = g.kw = 4
    g.sh = g.sw = g.dil = 1
    g.pt, g.pb, g.pl, g.pr = 2, 1, 2, 1
    g.OH, g.OW, g.T = h // 2, w // 2, 16
    return g


class StemS2dFn(torch.autograd.Function):
    """The ResNet stem conv on the space-to-depth input (the image itself needs no gradient)."""

    @staticmethod
    def forward(ctx, x, w, conv, want_stats, shift=None, s2d_hw=None):
        co = w.shape[0]
        if s2d_hw is not None:  # the loader converted the batch already (input_from_u8)
            n, (h, wd), xs = x.shape[0], s2d_hw, x
        else:
            n, _, h, wd = x.shape
            xs = _empty_cl(n, 16, h // 2, wd // 2, x.device)
            C.prepare_input_s2d(x.contiguous(), xs, n, h, wd)
        g = _s2d_geom(n, h, wd, co)
        idx = _s2d_index(x.device)
        wq = torch.zeros(co, 256, dtype=BF16, device=x.device)
        wq[:, idx] = weight_bf16(w).view(co, 147)
        grp = stat_groups(g.N * g.OH * g.OW)
        stats = ws(x.device).stats_buf(co, grp) if want_stats else None
        if STEM_DIRECT and co == 64:  # halo-tile direct kernel (csrc/stem.hip)
            y = _empty_cl(g.N, co, g.OH, g.OW, x.device)
            C.stem_conv(xs, wq, y, stats, grp, g.N, g.OH, g.OW, shift=shift if want_stats else None)
        else:
            y = conv_forward_raw(xs, None, g, stats=stats, wb=wq.view(-1), shift=shift if want_stats else None)
        ctx.g = g
        ctx.save_for_backward(xs, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, w = ctx.saved_tensors
        g = ctx.g
        dy = _cl(dy)
        dw = None
        if ctx.needs_input_grad[1]:
            m, ntot = g.N * g.OH * g.OW, g.T * g.Cx
            kps, splits, stages = _wgrad_plan(g, dy, xs, m, ntot)
            full = torch.zeros(g.Co * ntot, dtype=torch.float32, device=dy.device)
            idx = _s2d_index(dy.device)
            slot = arena_slot(w)
            dw = slot if slot is not None else grad_buffer(w, zero=False)

            # the last weight gradient of backward: on the compute stream (idle by then) it runs beside the
            # side stream's backlog instead of behind it (conv_wgrad_raw, padded-channel path)
            _wgrad_launch(dy, xs, full, g, m, ntot, kps, splits, stages)
            dw.permute(0, 2, 3, 1).reshape(g.Co, 147).copy_(full.view(g.Co, ntot)[:, idx])
        return None, dw, None, None, None, None


# ---------------------------------------------------------------------------
# depthwise convolution (EfficientNet)
# ---------------------------------------------------------------------------
class DwConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, conv, fuse_bwd=False):
        g = conv_geom(x, conv)
        wt = weight_bf16_t(w, g.Co, g.T, 1)
        y = _empty_cl(g.N, g.Co, g.OH, g.OW, x.device)
        C.dw_fwd(x, wt, y, None, g.N, g.H, g.W, g.Co, g.OH, g.OW, g.kh, g.kw, g.sh, g.sw, g.pt, g.pl)
        ctx.g = g
        # producer BN of x (this conv its only consumer): its backward reduce rides in the dgrad kernel
        link = getattr(x, "_imgcls_link", None) if fuse_bwd else None
        ctx.link = link if (link is not None and link.y is not None and link.res is None
                            and C.dw_dgrad_link_ok(g.kh, g.kw, g.sh, g.sw, g.pt, g.pl)) else None
        ctx.save_for_backward(x, w, wt)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, wt = ctx.saved_tensors
        g = ctx.g
        dy = _cl(dy)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _empty_cl(g.N, g.Co, g.H, g.W, x.device)
            link = ctx.link
            if link is not None and not link.done:
                grp = stat_groups(g.N * g.H * g.W)
                if DETERMINISTIC:  # one partial row per block: every address gets one contribution
                    grp = max(grp, C.dw_dgrad_link_blocks(g.N, g.H, g.W, g.Co, g.OH, g.OW, g.kh, g.sh))
                link.part = ws(dx.device).take_part(g.Co, grp)
                link.groups = grp
                C.dw_dgrad(dy, wt, dx, g.N, g.H, g.W, g.Co, g.OH, g.OW, g.kh, g.kw, g.sh, g.sw, g.pt, g.pl,
                           link.y, link.coef, link.part, grp, link.act)
                link.done = True  # dx holds dz; the producer BN skips its reduce
                if link.group is not None:
                    _syncbn_bwd_start(link)
            else:
                C.dw_dgrad(dy, wt, dx, g.N, g.H, g.W, g.Co, g.OH, g.OW, g.kh, g.kw, g.sh, g.sw, g.pt, g.pl)
        dw = None
        if ctx.needs_input_grad[1]:
            dw = grad_buffer(w, zero=False)  # dw_wgrad overwrites it (ordered column sum of partial rows)
            C.dw_wgrad(dy, x, dw, g.N, g.H, g.W, g.Co, g.OH, g.OW, g.kh, g.kw, g.sh, g.sw, g.pt, g.pl)
        return dx, dw, None, None


# ---------------------------------------------------------------------------
# BatchNorm (+ residual) (+ activation)
# ---------------------------------------------------------------------------
def _bn_coef(y, gamma, beta, bn, stats_ready, shift=None):
    """Batch (training) or running (eval) statistics of ``y`` -> coef [4, C] = scale, shift, mean, invstd.
    ``shift``: the pivot the partial sums are taken about (``stat_shift``; the producer used the same).
    Returns (coef, SyncBN group or None, all-reduced count tensor or None)."""
    dev = y.device
    n, c, h, w = y.shape
    rows = n * h * w
    coef = torch.empty(4 * c, dtype=torch.float32, device=dev)
    group = count_t = None
    if bn.training:
        grp = stat_groups(rows)
        part = ws(dev).stats_buf(c, grp)
        if not stats_ready:
            C.bn_stats(y, rows, c, part, grp, shift=shift)
        group = _sync_group(bn)
        mom = bn.momentum if bn.momentum is not None else 0.1
        track = bn.track_running_stats and bn.running_mean is not None
        rs = (bn.running_mean, bn.running_var, bn.num_batches_tracked) if track else (None, None, None)
        if group is None:  # one launch: partial rows -> coefficients + running stats
            C.bn_reduce_finalize(part, grp, c, float(rows), gamma, beta, *rs, mom, bn.eps, coef, shift=shift)
        else:
            pc = peer_channel(group, 0)
            from ..parallel import comm_timer
            with comm_timer.span("syncbn_fwd"):
                if pc is not None and c <= PEER_BN_MAX_C:  # one kernel: reduce + xGMI exchange + finalize
                    count_t = torch.empty(1, dtype=torch.float64, device=dev)
                    pc.comm.bn_fwd(part, grp, c, float(rows), gamma, beta, *rs, mom, bn.eps, coef, count_t,
                                   shift=shift)
                else:
                    sums = torch.empty(2 * c + 1, dtype=torch.float64, device=dev)
                    C.bn_partials(part, grp, c, sums, None, None, float(rows))  # + local count in the tail
                    stats_all_reduce_(sums, group)
                    count_t = sums[2 * c:]
                    C.bn_finalize(sums, count_t, float(rows), gamma, beta, *rs, mom, bn.eps, c, coef, shift=shift)
    else:
        if stats_ready:
            raise RuntimeError("eval-mode BN received fused statistics")
        C.bn_eval_coef(gamma, beta, bn.running_mean, bn.running_var, bn.eps, c, coef)
    return coef, group, count_t


def _bn_bwd_k(part, grp, c, rows, training, group, count_t, params, dev, coef=None, xa=None):
    """BN-backward partial rows -> (k [2, C] for bn_bwd_elemt, dgamma, dbeta); SyncBN all-reduces the sums.
    ``xa`` (with ``coef``): also the fused elementwise map [3][C] for ``XaLink`` consumers."""
    k = torch.empty(2 * c, dtype=torch.float32, device=dev)
    dgamma = grad_buffer(params[0], zero=False)
    dbeta = grad_buffer(params[1], zero=False)
    if training and group is None:  # one launch: partial rows -> dgamma, dbeta, k (+ the fused map)
        C.bn_reduce_bwd(part, grp, c, float(rows), dgamma, dbeta, k, coef=coef if xa is not None else None, xa=xa)
        return k, dgamma, dbeta
    pc = peer_channel(group, 0) if (training and group is not None) else None
    from ..parallel import comm_timer
    if pc is not None and count_t is not None and c <= PEER_BN_MAX_C:  # reduce + exchange + k in one kernel
        with comm_timer.span("syncbn_bwd"):
            pc.comm.bn_bwd(part, grp, c, count_t, dgamma, dbeta, k)
    else:
        sums = torch.empty(2 * c, dtype=torch.float64, device=dev)
        C.bn_partials(part, grp, c, sums, dgamma, dbeta)
        if group is not None:
            with comm_timer.span("syncbn_bwd"):
                stats_all_reduce_(sums, group)
        if training:
            C.bn_bwd_k(sums, count_t, float(rows), c, k)
        else:  # running statistics are constants: dy = scale * dz
            k.zero_()
    if xa is not None:
        C.bn_xa_coef(coef, k, c, xa)
    return k, dgamma, dbeta


# The residual BN's ReLU mask (1 bit per element, written by bn_apply) replaces the consumer dgrad epilogue's
# re-read of the residual when it recomputes z = bn(y) + res > 0: ~11 GB less per ResNet-50 b1024 step.
RELU_MASK = os.environ.get("IMGCLS_RELU_MASK", "1") == "1"


class BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, gamma, beta, res, bn, act, stats_ready, res_slot=None, link=None, cat=None, xa=None,
                shift=None, defer=None):
        dev = y.device
        n, c, h, w = y.shape
        rows = n * h * w
        a = ACT[act]
        coef, group, count_t = _bn_coef(y, gamma, beta, bn, stats_ready, shift)
        if defer is not None:
            # deferred (XfHold): the consuming conv applies act(bn(y)) itself; the output stands for
            # act(bn(y)) but holds y (autograd returns a view of the input)
            if res is not None or cat is not None or a > 1:
                raise RuntimeError("deferred BN output: no residual / concat slice, identity or ReLU only")
            defer.coef, defer.act = coef, a
            out = y
        elif cat is not None:  # write straight into this branch's channel slice of the concat output
            cbuf, idx = cat
            base = cbuf.ensure(n, h, w, dev)
            C.bn_apply(y, coef, res, base, rows, c, cbuf.total, cbuf.offs[idx], a)
            out = cbuf.part(idx, c)
        elif FP8_FWD and c % 128 == 0:  # the consuming conv reads an MX-FP8 copy: produce it here
            out = _empty_cl(n, c, h, w, dev)
            q = torch.empty(rows * c, dtype=FP8, device=dev)
            qs = torch.empty(rows * c // 32, dtype=torch.uint8, device=dev)
            mask = (torch.empty(rows * c // 8, dtype=torch.uint8, device=dev)
                    if RELU_MASK and res is not None and a == 1 and bn.training and link is not None else None)
            C.bn_apply(y, coef, res, out, rows, c, c, 0, a, q, qs, mask=mask)
            out._imgcls_mx = (q, qs, out._version)
            if link is not None:
                link.mask = mask
        else:
            out = _empty_cl(n, c, h, w, dev)
            # residual + ReLU in training: also the 1-bit ReLU mask, which the consuming conv's dgrad epilogue
            # reads instead of re-reading the residual (1/16 of its bytes, RELU_MASK)
            mask = (torch.empty(rows * c // 8, dtype=torch.uint8, device=dev)
                    if RELU_MASK and res is not None and a == 1 and bn.training and link is not None else None)
            C.bn_apply(y, coef, res, out, rows, c, c, 0, a, mask=mask)
            if link is not None:
                link.mask = mask
        ctx.act, ctx.group, ctx.rows, ctx.c = a, group, rows, c
        ctx.training = bn.training
        ctx.count_t = count_t
        ctx.res_slot = res_slot
        ctx.link = None
        if link is not None and bn.training:  # (grad mode is always off inside forward)
            link.y, link.coef, link.res, link.act = y, coef, res, a
            link.group, link.params, link.c, link.rows = group, (gamma, beta), c, rows
            link.count_t = count_t
            ctx.link = link
        ctx.has_res = res is not None
        ctx.params = (gamma, beta)
        ctx.xa = xa if bn.training else None
        ctx.save_for_backward(y, coef, res if res is not None else y)
        return out

    @staticmethod
    def backward(ctx, gout):  # (with ``defer`` too: gout is the gradient w.r.t. act(bn(y)))
        y, coef, res = ctx.saved_tensors
        res = res if ctx.has_res else None
        dev = y.device
        c, rows = ctx.c, ctx.rows
        ldg = channel_slice_stride(gout)  # a concat's gradient arrives as a channel slice: read in place
        g = gout if ldg else _cl(gout)
        link = ctx.link
        grp = stat_groups(rows)
        pending = None
        # fused backward: the producer 1x1 conv applies the elementwise map itself (XaLink); it needs dz
        # dense (not a concat slice) and the training-mode statistics
        xa = ctx.xa if (ctx.xa is not None and ctx.training) else None
        if link is not None and link.done:
            # the consuming conv's dgrad epilogue already produced dz and the partial sums
            part, dz = link.part, g
            grp = link.part_rows()
            FUSED_BWD_COUNT[0] += 1
            pending = link.pending
            link.y = link.coef = link.res = link.mask = link.part = link.pending = link.params = link.count_t = None
            if ldg:
                xa = None
        else:
            part = ws(dev).stats_buf(c, grp)
            if xa is not None and ldg:
                xa = None
            if ctx.has_res or (xa is not None and ctx.act != 0):
                dz = torch.empty_like(y, memory_format=CL)  # the residual's gradient and / or the fused input
            elif xa is not None:
                dz = g  # no activation: the incoming gradient is dz
            else:
                dz = None
            C.bn_bwd_reduce(g, y, coef, res, dz if dz is not g else None, rows, c, ctx.act, part, grp, ldg)
        xac = torch.empty(3 * c, dtype=torch.float32, device=dev) if xa is not None else None
        if pending is not None:  # SyncBN all-reduce launched early by the consuming conv's backward
            sums, work, dgamma, dbeta, k = pending
            work.wait()
            if k is None:
                k = torch.empty(2 * c, dtype=torch.float32, device=dev)
                C.bn_bwd_k(sums, ctx.count_t, float(rows), c, k)
            if xac is not None:
                C.bn_xa_coef(coef, k, c, xac)
        else:
            k, dgamma, dbeta = _bn_bwd_k(part, grp, c, rows, ctx.training, ctx.group, ctx.count_t, ctx.params, dev,
                                         coef=coef, xa=xac)
        if link is not None and link.done:
            ws(dev).give_part(part)
        if xa is not None:
            # hand dz and the map to the producer conv: no bn_bwd_elemt pass, no dY tensor
            xa.dz, xa.y, xa.coef = dz, y, xac
            XA_COUNT[0] += 1
            dy = dz
        else:
            dy = torch.empty_like(y, memory_format=CL)
            C.bn_bwd_elemt(None if dz is not None else g, y, coef, k, res, dz, dy, rows, c, ctx.act,
                           0 if dz is not None else ldg)
        dres = dz if ctx.has_res else None
        if dres is not None and ctx.res_slot is not None:
            dres = ctx.res_slot.deliver(dres)
        return dy, dgamma, dbeta, dres, None, None, None, None, None, None, None, None, None


class BNActPoolFn(torch.autograd.Function):
    """maxpool(act(BN(y))) for network stems (ResNet conv1 -> bn1 -> relu -> maxpool 3/2/1, Inception
    Conv2d_2b / Conv2d_4a -> maxpool 3/2/0).  The forward pools straight from ``y`` (the
    full-resolution activation is never written or re-read).  The backward is maxpool_bwd -> BN backward:
    gathering the pooled gradient inside both BN-backward passes measured slower (docs/DESIGN.md)."""

    @staticmethod
    def forward(ctx, y, gamma, beta, bn, act, stats_ready, pool, shift=None):
        dev = y.device
        n, c, h, w = y.shape
        (kh, kw), (sh, sw), (ph, pw) = pool
        oh = (h + 2 * ph - kh) // sh + 1
        ow = (w + 2 * pw - kw) // sw + 1
        a = ACT[act]
        coef, group, count_t = _bn_coef(y, gamma, beta, bn, stats_ready, shift)
        out = _empty_cl(n, c, oh, ow, dev)
        idx = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=dev)
        geo = [h, w, oh, ow, kh, kw, sh, sw, ph, pw]
        C.bn_act_maxpool(y, coef, out, idx, n, c, geo, a)
        ctx.act, ctx.group, ctx.count_t, ctx.geo = a, group, count_t, geo
        ctx.training = bn.training
        ctx.params = (gamma, beta)
        ctx.save_for_backward(y, coef, idx)
        return out

    @staticmethod
    def backward(ctx, gout):
        y, coef, idx = ctx.saved_tensors
        dev = y.device
        n, c, h, w = y.shape
        rows = n * h * w
        _, _, oh, ow, kh, kw, sh, sw, ph, pw = ctx.geo
        g = _empty_cl(n, c, h, w, dev)
        C.maxpool_bwd(_cl(gout), idx, g, n, h, w, c, oh, ow, kh, kw, sh, sw, ph, pw)
        grp = stat_groups(rows)
        part = ws(dev).stats_buf(c, grp)
        C.bn_bwd_reduce(g, y, coef, None, None, rows, c, ctx.act, part, grp)
        k, dgamma, dbeta = _bn_bwd_k(part, grp, c, rows, ctx.training, ctx.group, ctx.count_t, ctx.params, dev)
        dy = torch.empty_like(y, memory_format=CL)
        C.bn_bwd_elemt(g, y, coef, k, None, None, dy, rows, c, ctx.act)
        return dy, dgamma, dbeta, None, None, None, None, None


STEM_POOL_FUSE = os.environ.get("IMGCLS_STEM_POOL_FUSE", "1") == "1"


def conv_bn_act_pool(x, conv, bn, act, pool, exclusive_input=False):
    """max_pool2d(act(bn(conv(x))), *pool) with the pool fused into the BN passes (stems).
    ``exclusive_input`` as for ``conv_bn_act`` (the conv's dgrad may run x's producer BN reduce)."""
    x = materialize_deferred(x)
    k, s, p = _pool_args(*pool)
    if not STEM_POOL_FUSE or k[0] * k[1] > 255 or 2 * p[0] > k[0] or 2 * p[1] > k[1]:
        return max_pool2d(conv_bn_act(x, conv, bn, act, None, exclusive_input=exclusive_input), *pool)
    ensure_channels_last_weight(conv)
    shift = stat_shift(bn)
    if stem_s2d_eligible(x, conv) and not x.requires_grad:
        y = StemS2dFn.apply(x, conv.weight, conv, bn.training, shift, getattr(x, "_imgcls_s2d", None))
    else:
        if conv.groups != 1 or conv.bias is not None:
            raise NotImplementedError("conv_bn_act_pool: grouped conv / conv bias")
        y = ConvFn.apply(_cl(x), conv.weight, conv, bn.training, None, exclusive_input and FUSE_BN_BWD, None, shift)
    return BNActPoolFn.apply(y, bn.weight, bn.bias, bn, act, bn.training, (k, s, p), shift)


def dense_conv_eligible(x, conv) -> bool:
    """The kernel covers the whole unpadded input: one output pixel per image (a dense layer)."""
    return (x.dim() == 4 and tuple(x.shape[2:]) == tuple(conv.kernel_size) and conv.groups == 1
            and conv.bias is None and tuple(conv.padding) == (0, 0) and tuple(conv.dilation) == (1, 1)
            and not getattr(conv, "tf_same", False) and x.shape[1] == conv.in_channels)


def _dense_geom(n, k, co) -> ConvGeom:
    """A dense layer Y[n][co] = X[n][k] . W[co][k] as a 1x1 conv over a 1x1 map with k input channels."""
    g = ConvGeom.__new__(ConvGeom)
    g.taps = g.phases = None
    g.N, g.Ci, g.Cx, g.H, g.W, g.Co = n, k, k, 1, 1, co
    g.kh = g.kw = g.sh = g.sw = g.dil = 1
    g.pt = g.pb = g.pl = g.pr = 0
    g.OH = g.OW = g.T = 1
    return g


def _as_pixel_rows(t, n, k):
    """[n, c, h, w] channels-last -> [n, k = h*w*c, 1, 1] channels-last: the same memory, one 'pixel' per image."""
    return _cl(t).permute(0, 2, 3, 1).reshape(n, k).view(n, k, 1, 1)


class DenseConvFn(torch.autograd.Function):
    """A convolution whose kernel covers its whole unpadded input is a dense layer:
    Y[n][co] = X[n][(h, w, ci)] . W[co][(h, w, ci)] - NHWC activations and KRSC weights flatten alike
    (Inception's aux classifier conv1: 5x5 over a 5x5 map, reference nn/classifier.py:20-23 via
    torchvision's InceptionAux).  As an implicit-GEMM 5x5 conv its data gradient walked all 25 taps per
    input pixel, 24 of them in the zero padding (279 us of 64 blocks at batch 128).  Here it runs on the
    same MFMA implicit-GEMM kernels as a 1x1 conv over a 1x1 map with h*w*ci input channels: forward
    (with the following BN's statistics in the epilogue), data gradient (transposed bf16 shadow) and
    split-K weight gradient into the gradient arena slot - no library GEMM."""

    @staticmethod
    def forward(ctx, x, w, conv, want_stats=False, shift=None):
        n, c, h, wd = x.shape
        co = w.shape[0]
        k = h * wd * c
        g = _dense_geom(n, k, co)
        xf = _as_pixel_rows(x, n, k)
        stats = ws(x.device).stats_buf(co, stat_groups(n)) if want_stats else None
        y = conv_forward_raw(xf, w, g, stats=stats, wb=weight_bf16(w), shift=shift if want_stats else None)
        ctx.g, ctx.xshape = g, (n, c, h, wd)
        ctx.save_for_backward(xf, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        xf, w = ctx.saved_tensors
        g = ctx.g
        n, c, h, wd = ctx.xshape
        dy = _cl(dy)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            d = conv_dgrad_raw(dy, w, g)  # [n, k, 1, 1] channels-last = [n][h][w][c] in memory
            dx = torch.empty(0, dtype=d.dtype, device=d.device).set_(
                d.untyped_storage(), d.storage_offset(), (n, c, h, wd), (h * wd * c, 1, wd * c, c))
        if ctx.needs_input_grad[1]:
            dw = conv_wgrad_raw(dy, xf, w, g)
        return dx, dw, None, None, None


POOL_CONV_SWAP = os.environ.get("IMGCLS_POOL_CONV_SWAP", "1") == "1"


def pool_conv_bn_act(x, conv, bn, act, prepool, x_slot=None, out=None, out_plan=None):
    """act(bn(conv(avg_pool2d(x, *prepool)))) (count_include_pad pooling).  A 1x1 stride-1 conv commutes
    with the pool, so the conv runs first and the pool moves the conv's output: the Inception
    ``branch_pool`` convs narrow 192-2048 channels to 32-192, so the pool's forward and backward passes
    move 4-11x fewer bytes, and the conv's dgrad (not an avgpool backward) delivers into the block
    input's gradient slot.  BN statistics are taken after the pool."""
    x = materialize_deferred(x)
    k, s, p = _pool_args(*prepool)
    pointwise = (tuple(conv.kernel_size) == (1, 1) and tuple(conv.stride) == (1, 1)
                 and tuple(conv.padding) == (0, 0) and conv.groups == 1 and conv.bias is None
                 and not getattr(conv, "tf_same", False))
    if not (POOL_CONV_SWAP and pointwise):
        from .functional import conv_bn_act as _f_conv_bn_act
        return _f_conv_bn_act(avg_pool2d(x, *prepool, slot=x_slot), conv, bn, act, out=out_plan)
    x = _cl(x)
    ensure_channels_last_weight(conv)
    y = ConvFn.apply(x, conv.weight, conv, False, x_slot, False)
    yp = AvgPoolFn.apply(y, k, s, p, None)
    return BNActFn.apply(yp, bn.weight, bn.bias, None, bn, act, False, None, None, out, None, stat_shift(bn))


def conv_bn_act(x, conv, bn, act, residual, x_slot=None, res_slot=None, exclusive_input=False, out=None,
                defer_act=False):
    """``exclusive_input``: this conv is the only consumer of ``x`` (lets its dgrad fuse the BN-backward
    reduce of x's producer); a slot-paired consumer qualifies automatically.  ``out`` = (ConcatBuffer,
    branch index): the result is written into that branch's channel slice of the concat output.
    ``defer_act``: the result only feeds the next ``conv_bn_act`` (as its exclusive input); in training the
    BN then hands that conv y and its map instead of writing act(bn(y)) (``XfHold``)."""
    shift = stat_shift(bn)
    xf = getattr(x, "_imgcls_xf", None)
    if xf is not None and not xf_eligible(x, conv):
        x, xf = XfMaterializeFn.apply(x, xf), None
    if stem_s2d_eligible(x, conv) and residual is None and not x.requires_grad:
        ensure_channels_last_weight(conv)
        y = StemS2dFn.apply(x, conv.weight, conv, bn.training, shift, getattr(x, "_imgcls_s2d", None))
        link = BwdLink() if (FUSE_BN_BWD and bn.training and torch.is_grad_enabled()) else None
        out = BNActFn.apply(y, bn.weight, bn.bias, None, bn, act, bn.training, None, link, None, None, shift)
        if link is not None:
            out._imgcls_link = link
        return out
    x = _cl(x)
    if residual is not None:
        residual = _cl(residual)
    ensure_channels_last_weight(conv)
    depthwise = conv.groups > 1
    dense = False
    xa = None
    if depthwise:
        if not (conv.groups == conv.in_channels == conv.out_channels):
            raise NotImplementedError("grouped (non-depthwise) convolution")
        y = DwConvFn.apply(x, conv.weight, conv, exclusive_input and FUSE_BN_BWD and DW_LINK)
        ready = False
    elif dense_conv_eligible(x, conv) and x.shape[2] * x.shape[3] > 1:
        dense = True
        y = DenseConvFn.apply(x, conv.weight, conv, bn.training, shift)
        ready = bn.training
    else:
        if conv.groups != 1:
            raise NotImplementedError("grouped convolution")
        xa = XaLink() if (bn.training and torch.is_grad_enabled() and xa_eligible(x, conv)) else None
        y = ConvFn.apply(x, conv.weight, conv, bn.training, x_slot, exclusive_input and FUSE_BN_BWD, xa, shift, xf)
        xf = None
        ready = bn.training
    if xf is not None:
        raise RuntimeError("deferred BN output reached a consumer without the fused map")
    if conv.bias is not None:
        raise NotImplementedError("conv bias before BatchNorm")
    link = BwdLink() if (FUSE_BN_BWD and bn.training and torch.is_grad_enabled()) else None
    hold = XfHold() if (defer_act and FUSE_XF and bn.training and torch.is_grad_enabled() and residual is None
                        and out is None and ACT[act] <= 1 and not FP8_FWD) else None
    res_out = BNActFn.apply(y, bn.weight, bn.bias, residual, bn, act, ready, res_slot, link, out,
                            xa if not depthwise and not dense else None, shift, hold)
    if link is not None:
        res_out._imgcls_link = link
    if hold is not None:
        res_out._imgcls_xf = hold
    return res_out


class ConvBiasFn(torch.autograd.Function):
    """Plain convolution with optional bias (no BN)."""

    @staticmethod
    def forward(ctx, x, w, b, conv):
        g = conv_geom(x, conv)
        y = conv_forward_raw(x, w, g, bias=b)
        ctx.g = g
        ctx.has_b = b is not None
        ctx.bias = b
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        g = ctx.g
        dy = _cl(dy)
        dx = conv_dgrad_raw(dy, w, g) if ctx.needs_input_grad[0] else None
        dw = conv_wgrad_raw(dy, x, w, g) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            grp = stat_groups(g.N * g.OH * g.OW)
            part = ws(dy.device).stats_buf(g.Co, grp)
            C.bn_stats(dy, g.N * g.OH * g.OW, g.Co, part, grp)
            sums = torch.empty(2 * g.Co, dtype=torch.float64, device=dy.device)
            db = grad_buffer(ctx.bias, zero=False)
            C.bn_partials(part, grp, g.Co, sums, None, db)
        return dx, dw, db, None


def conv(x, conv_mod):
    ensure_channels_last_weight(conv_mod)
    if conv_mod.groups != 1:
        raise NotImplementedError("grouped convolution without BN")
    return ConvBiasFn.apply(_cl(x), conv_mod.weight, conv_mod.bias, conv_mod)


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


# ---------------------------------------------------------------------------
# classifier head (fp32)
# ---------------------------------------------------------------------------
def _mm(a, b, out, m, n, k, sam, sak, sbk, sbn, bias=None, mask=None, smm=0, smk=0, relu=False, acc=False):
    C.sgemm(a, b, out, bias, mask, m, n, k, sam, sak, sbk, sbn, n if out.dim() == 2 else out.stride(0),
            smm, smk, relu, acc)


class MlpFn(torch.autograd.Function):
    """Stack of Linear layers, ReLU after every layer whose flag is set."""

    @staticmethod
    def forward(ctx, x, relus, *wb):
        x = x.contiguous().float()
        acts = [x]
        h = x
        for i, r in enumerate(relus):
            w, b = wb[2 * i], wb[2 * i + 1]
            nout, nin = w.shape
            y = torch.empty((h.shape[0], nout), dtype=torch.float32, device=h.device)
            _mm(h, w.contiguous(), y, h.shape[0], nout, nin, nin, 1, 1, nin, bias=b, relu=r)
            acts.append(y)
            h = y
        ctx.relus = relus
        ctx.params = wb
        ctx.nb = [b is not None for b in wb[1::2]]
        ctx.save_for_backward(*acts, *[w for w in wb[0::2]])
        return h

    @staticmethod
    def backward(ctx, gout):
        saved = ctx.saved_tensors
        nl = len(ctx.relus)
        acts, ws_ = saved[:nl + 1], saved[nl + 1:]
        g = gout.contiguous().float()
        grads = [None] * (2 * nl)
        mb = g.shape[0]
        for i in reversed(range(nl)):
            w = ws_[i].contiguous()
            nout, nin = w.shape
            xin, yout = acts[i], acts[i + 1]
            mask = yout if ctx.relus[i] else None
            dw = grad_buffer(ctx.params[2 * i], zero=False)
            # dW[o][f] = sum_b g[b][o] * x[b][f]   (A(m=o,k=b) = g[b][o])
            _mm(g, xin, dw, nout, nin, mb, 1, nout, nin, 1, mask=mask, smm=1, smk=nout)
            grads[2 * i] = dw
            if ctx.nb[i]:
                db = grad_buffer(ctx.params[2 * i + 1], zero=False)
                C.colsum(g, mask, db, mb, nout, nout, False)
                grads[2 * i + 1] = db
            if i > 0 or ctx.needs_input_grad[0]:
                dx = torch.empty((mb, nin), dtype=torch.float32, device=g.device)
                # dX[b][f] = sum_o g[b][o] * W[o][f]
                _mm(g, w, dx, mb, nin, nout, nout, 1, nin, 1, mask=mask, smm=nout, smk=1)
                g = dx
        return (g if ctx.needs_input_grad[0] else None, None, *grads)


def mlp(x, seq):
    import torch.nn as nn
    layers = list(seq) if isinstance(seq, nn.Sequential) else [seq]
    lins, relus = [], []
    for m in layers:
        if isinstance(m, nn.Linear):
            lins.append(m)
            relus.append(False)
        elif isinstance(m, nn.ReLU):
            relus[-1] = True
        else:
            raise NotImplementedError(f"head layer {type(m).__name__}")
    wb = []
    for m in lins:
        wb += [m.weight, m.bias]
    return MlpFn.apply(x, tuple(relus), *wb)


def linear(x, lin, act=None):
    if act not in (None, "relu"):
        raise NotImplementedError(act)
    return MlpFn.apply(x, (act == "relu",), lin.weight, lin.bias)


class CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, weight):
        x = logits.contiguous().float()
        b, c = x.shape
        prob = torch.empty_like(x)
        out = torch.empty(2, dtype=torch.float32, device=x.device)
        lab = labels.contiguous().long()
        C.ce_fwd(x, lab, weight, prob, out, b, c)
        ctx.save_for_backward(prob, lab, out, weight if weight is not None else out)
        ctx.has_w = weight is not None
        return out[0]

    @staticmethod
    def backward(ctx, gout):
        prob, lab, out, w = ctx.saved_tensors
        b, c = prob.shape
        dx = torch.empty_like(prob)
        C.ce_bwd(prob, lab, w if ctx.has_w else None, out, gout.reshape(1).float().contiguous(), dx, b, c)
        return dx, None, None


def cross_entropy(logits, labels, weight=None):
    return CrossEntropyFn.apply(logits, labels, weight)


# ---------------------------------------------------------------------------
# misc
# ---------------------------------------------------------------------------
_AFFINE_CACHE: dict = {}


def prepare_input(x, scale=None, shift=None, stem=None):
    """fp32 NCHW batch -> bf16 NHWC padded to a multiple of 8 channels (one kernel).  With ``stem``
    (the first conv) eligible for the space-to-depth form, the fp32 batch is returned unchanged: the
    stem converts it itself (``StemS2dFn``)."""
    if getattr(x, "_imgcls_s2d", None) is not None:
        if stem is None or scale is not None or not stem_s2d_eligible(x, stem):
            raise ValueError("a space-to-depth input batch (input_from_u8) reached a model without the s2d stem")
        return x
    if getattr(x, "_imgcls_prepared", False):
        return x  # converted by the loader, the model's affine included (input_from_u8)
    if stem is not None and scale is None and stem_s2d_eligible(x, stem):
        return x
    if x.dtype == BF16 and x.is_contiguous(memory_format=CL) and x.shape[1] % 8 == 0:
        return x
    x = x.contiguous().float()
    n, c, h, w = x.shape
    cp = (c + 7) // 8 * 8
    y = _empty_cl(n, cp, h, w, x.device)
    sc = sh = None
    if scale is not None:
        key = (x.device, tuple(scale), tuple(shift))
        if key not in _AFFINE_CACHE:
            _AFFINE_CACHE[key] = (torch.tensor(scale, dtype=torch.float32, device=x.device),
                                  torch.tensor(shift, dtype=torch.float32, device=x.device))
        sc, sh = _AFFINE_CACHE[key]
    C.prepare_input(x, y, n, c, h * w, cp, sc, sh)
    return y


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


CONCAT_INPLACE = os.environ.get("IMGCLS_CONCAT_INPLACE", "1") == "1"  # 0: copy branches into the concat


class ConcatBuffer:
    """Output of a channel concat (Inception blocks) that the branches write in place:
    each branch's final BN-apply stores straight into its channel slice (``conv_bn_act(out=(buf, i))``),
    ``cat_channels(parts, buf)`` then only copies branches that were produced elsewhere (pools), and its
    backward hands every in-place branch its gradient slice without a copy (BN backward reads it with
    a row stride).  Allocated lazily by the first branch (which knows the batch and spatial size)."""

    def __init__(self, channels):
        self.cs = list(channels)
        self.offs = [sum(self.cs[:i]) for i in range(len(self.cs))]
        self.total = sum(self.cs)
        self.buf = None
        self.ptrs = [None] * len(self.cs)

    def ensure(self, n, h, w, dev):
        if self.buf is None:
            self.buf = _empty_cl(n, self.total, h, w, dev)
        elif tuple(self.buf.shape) != (n, self.total, h, w):
            raise RuntimeError("concat branches disagree on the output shape")
        return self.buf

    def part(self, i, c):
        """Branch i's slice as a tensor sharing the buffer's storage but not an autograd view of it
        (several custom Functions write into one base; views would trip autograd's view+inplace check)."""
        if c != self.cs[i]:
            raise RuntimeError(f"concat branch {i}: {c} channels, planned {self.cs[i]}")
        b = self.buf
        n, _, h, w = b.shape
        t = torch.empty(0, dtype=b.dtype, device=b.device)
        t.set_(b.untyped_storage(), b.storage_offset() + self.offs[i], (n, c, h, w),
               (h * w * self.total, 1, w * self.total, self.total))
        self.ptrs[i] = t.data_ptr()
        return t


class CatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cbuf, *xs):
        n, _, h, w = xs[0].shape
        cs = [t.shape[1] for t in xs]
        if cbuf is None:
            cbuf = ConcatBuffer(cs)
        elif cs != cbuf.cs:
            raise RuntimeError(f"cat_channels: parts {cs} != planned {cbuf.cs}")
        y = cbuf.ensure(n, h, w, xs[0].device)
        rows = n * h * w
        inplace = []
        for i, (t, c) in enumerate(zip(xs, cs)):
            done = cbuf.ptrs[i] is not None and t.data_ptr() == cbuf.ptrs[i]
            if not done:
                C.copy_channels(_cl(t), c, 0, y, cbuf.total, cbuf.offs[i], rows, c)
            inplace.append(done)
        ctx.cs, ctx.inplace = cs, inplace
        ctx.geo = (n, h, w)
        return y

    @staticmethod
    def backward(ctx, gy):
        gy = _cl(gy)
        n, h, w = ctx.geo
        tot = sum(ctx.cs)
        outs, off = [], 0
        for c, inplace in zip(ctx.cs, ctx.inplace):
            if inplace:  # BN backward reads the slice in place (row stride tot)
                outs.append(gy[:, off:off + c])
            else:
                g = _empty_cl(n, c, h, w, gy.device)
                C.copy_channels(gy, tot, off, g, c, 0, n * h * w, c)
                outs.append(g)
            off += c
        return (None,) + tuple(outs)


def cat_channels(xs, buf=None):
    return CatFn.apply(buf, *xs)


class AddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        y = torch.empty_like(a, memory_format=CL)
        C.add(a, b, y)
        return y

    @staticmethod
    def backward(ctx, g):
        return g, g


def add(x, y):
    return AddFn.apply(_cl(x), _cl(y))


class DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        x = x.contiguous().float()
        seed = torch.randint(0, 2**31 - 1, (2,), device=x.device, dtype=torch.int64)
        y = torch.empty_like(x)
        mask = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
        C.dropout(x, y, mask, p, seed)
        ctx.p = p
        ctx.save_for_backward(mask)
        return y

    @staticmethod
    def backward(ctx, g):
        (mask,) = ctx.saved_tensors
        dx = torch.empty_like(mask, dtype=torch.float32)
        C.dropout_bwd(g.contiguous().float(), mask, dx, ctx.p)
        return dx, None


def dropout(x, p):
    return DropoutFn.apply(x, float(p))


class ScaleRowsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale):
        y = torch.empty_like(x, memory_format=CL)
        per = x.numel() // x.shape[0]
        C.scale_rows(x, scale, y, per)
        ctx.save_for_backward(scale)
        ctx.per = per
        return y

    @staticmethod
    def backward(ctx, g):
        (scale,) = ctx.saved_tensors
        g = _cl(g)
        dx = torch.empty_like(g, memory_format=CL)
        C.scale_rows(g, scale, dx, ctx.per)
        return dx, None


def drop_connect(x, p):
    keep = 1.0 - p
    r = torch.rand(x.shape[0], dtype=torch.float32, device=x.device)
    scale = torch.floor(r + keep) / keep
    return ScaleRowsFn.apply(_cl(x), scale)


# depthwise dgrad runs its producer BN's backward reduce: measured 0.6 % slower on EfficientNet-B0 (the extra
# y loads and coefficients lift the row-strip kernels to 2 waves per SIMD), so opt-in
DW_LINK = os.environ.get("IMGCLS_DW_LINK", "0") == "1"
SE_FUSED = os.environ.get("IMGCLS_SE_FUSED", "1") == "1"  # csrc/se.hip MLP kernels (0: GEMM + activation launches)


class SEFn(torch.autograd.Function):
    """Squeeze-excitation gate y = x * sigmoid(W_e silu(W_r mean_hw(x) + b_r) + b_e) (efficientnet_pytorch
    MBConvBlock).  Fused path: spatial mean -> one MLP kernel -> scale (forward); spatial dot -> per-image
    MLP backward -> weight gradients -> dx (backward)."""

    @staticmethod
    def forward(ctx, x, wr, br, we, be, fuse_bwd=False):
        n, c, h, w = x.shape
        hw = h * w
        # producer BN of x (the gate is x's only consumer): its backward reduce rides in se_dx
        link = getattr(x, "_imgcls_link", None) if fuse_bwd else None
        ctx.link = link if (link is not None and link.y is not None and link.res is None) else None
        nsq = wr.shape[0]
        wr2, we2 = wr.reshape(nsq, c).contiguous(), we.reshape(c, nsq).contiguous()
        p = torch.empty((n, c), dtype=torch.float32, device=x.device)
        C.gap_fwd(x, p, n, hw, c)
        fused = SE_FUSED and br is not None and be is not None and nsq <= 160
        hpre = torch.empty((n, nsq), dtype=torch.float32, device=x.device)
        s = torch.empty((n, c), dtype=torch.float32, device=x.device)
        if fused:
            we2 = we2.t().contiguous()  # W_e^T [nsq][C]: channel-contiguous weight reads in both kernels
            C.se_mlp_fwd(p, wr2, br.contiguous(), we2, be.contiguous(), hpre, s, n, c, nsq)
            a = hpre  # (unused by the fused backward, which recomputes silu(h))
        else:
            _mm(p, wr2, hpre, n, nsq, c, c, 1, 1, c, bias=br)
            a = torch.empty_like(hpre)
            C.act32_fwd(hpre, a, 0)
            e = torch.empty((n, c), dtype=torch.float32, device=x.device)
            _mm(a, we2, e, n, c, nsq, nsq, 1, 1, nsq, bias=be)
            C.act32_fwd(e, s, 1)
        y = torch.empty_like(x, memory_format=CL)
        C.se_scale(x, s, y, n, hw, c)
        ctx.save_for_backward(x, p, hpre, a, s, wr2, we2)
        ctx.geo = (n, c, hw, nsq)
        ctx.params = (wr, br, we, be)
        ctx.fused = fused
        return y

    @staticmethod
    def backward(ctx, dy):
        x, p, hpre, a, s, wr2, we2 = ctx.saved_tensors
        n, c, hw, nsq = ctx.geo
        dy = _cl(dy)
        dev = dy.device
        ds = torch.empty((n, c), dtype=torch.float32, device=dev)
        C.se_ds(dy, x, ds, n, hw, c)
        wr, br, we, be = ctx.params
        dwe = grad_buffer(we, zero=False)  # [c][nsq](1x1) in memory for either weight layout
        dbe = grad_buffer(be, zero=False)
        dwr = grad_buffer(wr, zero=False)
        dbr = grad_buffer(br, zero=False)
        dp = torch.empty((n, c), dtype=torch.float32, device=dev)
        if ctx.fused:
            de = torch.empty_like(ds)
            dh = torch.empty((n, nsq), dtype=torch.float32, device=dev)
            C.se_mlp_bwd(ds, s, hpre, p, wr2, we2, de, dh, dp, dwr, dbr, dwe, dbe, n, c, nsq)
        else:
            de = torch.empty_like(ds)
            C.act32_bwd(s, ds, de, 2)
            _mm(de, a, dwe, c, nsq, n, 1, c, nsq, 1)
            C.colsum(de, None, dbe, n, c, c, False)
            da = torch.empty((n, nsq), dtype=torch.float32, device=dev)
            _mm(de, we2, da, n, nsq, c, c, 1, nsq, 1)
            dh = torch.empty_like(da)
            C.act32_bwd(hpre, da, dh, 0)
            _mm(dh, p, dwr, nsq, c, n, 1, nsq, c, 1)
            C.colsum(dh, None, dbr, n, nsq, nsq, False)
            _mm(dh, wr2, dp, n, c, nsq, nsq, 1, c, 1)
        dx = torch.empty_like(dy, memory_format=CL)
        link = ctx.link
        if link is not None and not link.done:
            grp = C.se_dx_link_blocks(n, hw, c)  # one partial row per block, plain stores (no atomics)
            link.part = ws(dev).take_part(c, grp)
            link.groups = grp
            C.se_dx(dy, s, dp, dx, n, hw, c, link.y, link.coef, link.part, grp, link.act)
            link.done = True  # dx holds dz; the producer BN skips its reduce
            if link.group is not None:
                _syncbn_bwd_start(link)
        else:
            C.se_dx(dy, s, dp, dx, n, hw, c)
        return dx, dwr, dbr, dwe, dbe, None


SE_LINK = os.environ.get("IMGCLS_SE_LINK", "1") == "1"  # se_dx runs the gate input's producer BN backward reduce


def se_gate(x, se_reduce, se_expand, exclusive_input=False):
    """``exclusive_input``: the gate is x's only consumer (x = act(BN(y)) in an MBConv block), so its
    backward may emit dz and the producer BN's partial sums."""
    return SEFn.apply(_cl(x), se_reduce.weight, se_reduce.bias, se_expand.weight, se_expand.bias,
                      exclusive_input and FUSE_BN_BWD and SE_LINK)


# ---------------------------------------------------------------------------
# fused Adam
# ---------------------------------------------------------------------------
_ADAM_CHUNK = 65536
_TENSOR_DT = np.dtype([("p", "<u8"), ("g", "<u8"), ("m", "<u8"), ("v", "<u8"), ("s", "<u8"), ("n", "<i8")])
_WTJOB_DT = np.dtype([("w", "<u8"), ("o", "<u8"), ("co", "<i4"), ("t", "<i4"), ("ci", "<i4"), ("pad", "<i4")])


def _upload(arr: np.ndarray, dev) -> torch.Tensor:
    # pinned + non_blocking: a pageable H2D copy would stall the host until the GPU drains
    return torch.from_numpy(arr).pin_memory().to(dev, non_blocking=True)


def _same_memory_order(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Dense tensors whose elements sit in the same order in memory (size-1 dims ignored)."""
    if a.shape != b.shape:
        return False
    dense = lambda t: t.is_contiguous() or t.is_contiguous(memory_format=CL)  # noqa: E731
    if not (dense(a) and dense(b)):
        return False
    return all(sa == sb for n, sa, sb in zip(a.shape, a.stride(), b.stride()) if n > 1)


def adam_build_table(opt, items):
    if C.weight_t_job_bytes() != _WTJOB_DT.itemsize:
        raise RuntimeError("weight_t_tiles: job record layout mismatch between Python and the kernel")
    groups = {}
    wt_jobs = []
    mx_jobs = []
    for gi, group, p in items:
        groups.setdefault(gi, (group, []))[1].append(p)
    tables = []
    for gi, (group, ps) in sorted(groups.items()):
        recs = np.zeros(len(ps), dtype=_TENSOR_DT)
        chunks = []
        for t, p in enumerate(ps):
            st = opt.state[p]
            sh = shadow_for_optimizer(p)
            recs[t] = (p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                       sh.data_ptr() if sh is not None else 0, p.numel())
            stt = shadow_t_for_optimizer(p) if sh is not None else None
            if stt is not None:
                wt_jobs.append((sh.data_ptr(), stt[0].data_ptr()) + tuple(stt[1:]) + (0,))
            smx = shadow_mx_for_optimizer(p) if sh is not None else None
            if smx is not None:
                mx_jobs.append((p.data_ptr(), smx[0].data_ptr(), smx[1].data_ptr(), p.numel()))
            for ck in range(-(-p.numel() // _ADAM_CHUNK)):
                chunks.append((t, ck))
            if not _same_memory_order(p, p.grad):
                raise RuntimeError("fused Adam: gradient layout differs from parameter layout")
        dev = ps[0].device
        tab = _upload(recs.view(np.uint8).copy(), dev)
        ck = _upload(np.asarray(chunks, dtype=np.int32).reshape(-1), dev)
        lr_step = getattr(opt, "_lr_step", {}).get(gi)
        if lr_step is None:
            step0 = float(opt.state[ps[0]]["step"]) if "step" in opt.state[ps[0]] else 0.0
            lr_step = torch.tensor([group["lr"], step0], dtype=torch.float32, device=dev)
            opt.__dict__.setdefault("_lr_step", {})[gi] = lr_step
        tables.append((gi, tab, ck, len(chunks), lr_step, [p for p in ps]))
    wt = None
    if wt_jobs:
        jobs = np.array(wt_jobs, dtype=_WTJOB_DT)
        tiles = [(j, t, co0, ci0) for j, (_w, _o, co, taps, ci, _p) in enumerate(wt_jobs)
                 for t in range(taps) for co0 in range(0, co, 64) for ci0 in range(0, ci, 64)]
        wt = (_upload(jobs.view(np.uint8).copy(), tables[0][1].device),
              _upload(np.asarray(tiles, dtype=np.int32).reshape(-1), tables[0][1].device), len(tiles))
    mx = None
    if mx_jobs:
        dev0 = tables[0][1].device
        tiles = _mx_tiles(mx_jobs)
        mx = (_upload(np.array(mx_jobs, dtype=_MXW_DT).view(np.uint8).copy(), dev0),
              _upload(np.asarray(tiles, dtype=np.int32).reshape(-1), dev0), len(tiles))
    return (tables, shadow_generation(), wt, mx)


def adam_step(opt, items, table, grad_scale):
    tables, gen, wt, mx = table
    if gen != shadow_generation():
        opt._table_key = None  # rebuild next step so new shadows are kept fresh
    for gi, tab, ck, nck, lr_step, ps in tables:
        group = opt.param_groups[gi]
        b1, b2 = group["betas"]
        C.adam_tick(lr_step, float(group["lr"]))
        C.adam(tab, ck, nck, lr_step, b1, b2, group["eps"], group["weight_decay"], float(grad_scale), _ADAM_CHUNK)
    if wt is not None:  # refresh every transposed dgrad shadow from the updated KRSC shadows: one launch
        C.weight_t_tiles(*wt)
    if mx is not None:  # and every MX-FP8 forward copy from the updated fp32 masters: one launch
        C.mx_quant_w(*mx)
    opt._host_steps = getattr(opt, "_host_steps", 0) + 1
