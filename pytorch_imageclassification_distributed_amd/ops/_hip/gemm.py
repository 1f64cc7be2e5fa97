"""Implicit-GEMM convolution launchers on MFMA (forward, data gradient, fused XA backward, weight
gradient) and the per-shape kernel tuner with its find-db (``save_tuning`` / ``load_tuning``).

Split out of ``ops/hip.py`` (the facade that re-exports every name here).
"""
from __future__ import annotations

import os

import torch

from ..grad_arena import arena_slot, grad_buffer
from . import common as _common
from . import shadows as _shadows
from .common import BF16, C, G_STATS, _empty_cl, _pad_tuple, stat_groups, ws
from .shadows import act_mx, weight_bf16, weight_bf16_t, weight_mx


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
        # a family switched off by its flag is not served from the db either, and the deep kernel's
        # diagnostic variants (var & 6: wrong results by design) and untuned ones (var & 256) never are
        if v[2] >= PW_BASE:
            ok = PW_CONV and not fp8 and v[2] - PW_BASE < len(conv_pw_cfgs()) and len(v) == 3
        elif v[2] >= DEEP_BASE:
            ok = (DEEP_CONV and not fp8 and v[2] - DEEP_BASE < len(conv_deep_cfgs()) and len(v) == 3
                  and not conv_deep_cfgs()[v[2] - DEEP_BASE][4] & (6 | 256))
        elif v[2] >= HALO_BASE:
            ok = HALO_CONV and not fp8 and v[2] - HALO_BASE < len(conv_halo_cfgs()) and len(v) == 3
        elif v[2] >= DIRECT_BASE:
            ok = DIRECT_CONV and v[2] - DIRECT_BASE in DIRECT_CFGS and len(v) == 3
        else:
            ok = v[2] < (nfp8 if fp8 else ncfg) and len(v) == 3
        if ok and k not in _STAGES_TUNED:
            _STAGES_TUNED[k] = v
            n += 1
    for ks, v in db.get("wgrad", []):
        try:
            k, v = ast.literal_eval(ks), tuple(int(x) for x in v)
        except (ValueError, SyntaxError, TypeError):
            continue
        if len(v) == 2 and 1 <= v[1] <= 15 and v[0] > 0 and k not in _WGRAD_TUNED and (WGRAD_DEEP or v[1] < 13):
            _WGRAD_TUNED[k] = v
            n += 1
    return n
CONV_FORCE_CFG = None  # (stages, tile_n, cfg) for every bf16 fwd/dgrad launch (tests)
CONV_FORCE_FP8_CFG = None  # (stages, tile_n, cfg) for every MX-FP8 forward launch (tests)
TUNE_LOG: list = []  # (M, Ncols, K, {cfg: ms}) per tuned geometry (benchmarks/conv_bench.py prints it)


def _conv_gemm(A, B, out, stats, bias, geo, dh, dw, tb, zero, addend=None, bwd=(None, None, None, None, 0, 1),
               groups=G_STATS, scales=(None, None), xa=None, shift=None, xf=None, mask=None, y2=None):
    """One implicit-GEMM launch.  The kernel configuration - LDS-DMA ring depth (1 = high occupancy,
    2 / 3 = pipelined) x output-channel tile (64 / 128 / 256: more tiles balance 256 CUs better on
    small layers) x pixel tile (128 rows on 4 waves, or 256 rows on 8 waves) - is chosen once per
    GEMM geometry by timing the candidates on scratch outputs (a conv-algorithm "find" step).
    ``xa`` = (y, coef [3][CA]): A holds a BN's pre-elementwise gradient dz and the kernel applies the
    BN backward's elementwise map on its operand loads (1x1 stride-1 geometry; ``XaLink``).
    ``xf`` = (coef, act): A holds a BN's input y and the kernel applies act(bn(y)) on its operand loads
    (``XfHold``).  ``y2`` = (y2, coef2, part2) with the masked BN-backward epilogue: the partial sums of a second
    BN that receives the same dz (a deferred downsample BN, ``BwdLink.ds``)."""
    y2k = dict(bwd_y2=y2[0], bwd_coef2=y2[1], bwd_part2=y2[2]) if y2 is not None else {}
    xa3 = (xa[0], xa[1], xa[2] if len(xa) > 2 else None) if xa is not None else (None, None, None)
    xf2 = (xf[0], xf[1]) if xf is not None else (None, 0)
    fused = xa is not None or xf is not None
    if DIRECT_FORCE is not None and not fused and y2 is None and \
            _direct_geom(geo, dh, dw, tb, out, bias, addend, bwd, scales) is not None and \
            _direct_variant_ok(DIRECT_FORCE, _direct_geom(geo, dh, dw, tb, out, bias, addend, bwd, scales)):
        cfg = (0, 0, DIRECT_BASE + DIRECT_FORCE)  # (tests) every eligible launch on this direct variant
    elif PW_FORCE is not None and not fused and scales[0] is None and bias is None and addend is None and \
            bwd[0] is None and bwd[1] is None and mask is None and _pw_ok(geo, dh, dw, tb) and \
            geo[2] <= conv_pw_cfgs()[PW_FORCE][1]:
        cfg = (0, 0, PW_BASE + PW_FORCE)  # (tests) every eligible launch on this pointwise variant
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
               DIRECT_CONV) + ((True,) if xa is not None else ()) + (("xf",) if xf is not None else ()) + \
            (("y2",) if y2 is not None else ())
        cfg = _STAGES_TUNED.get(key)
        if cfg is None:
            # (deterministic mode: a find-db entry or the shape heuristic, never a timing - timed picks differ
            # between processes, and different kernels round differently)
            cfg = (0, 0, -1) if (torch.cuda.is_current_stream_capturing() or _common.DETERMINISTIC) else _tune_conv(
                A, B, out, stats, bias, geo, dh, dw, tb, zero, addend, bwd, groups, scales, xa, xf, mask, y2)
            if cfg[0] or cfg[2] >= 0:
                _STAGES_TUNED[key] = cfg
    if cfg[2] >= PW_BASE:
        PW_COUNT[0] += 1
    elif cfg[2] >= DEEP_BASE:
        DEEP_COUNT[0] += 1
    elif cfg[2] >= HALO_BASE:
        HALO_COUNT[0] += 1
    elif cfg[2] >= DIRECT_BASE:
        if y2 is not None:
            raise RuntimeError("conv_gemm: the direct kernel has no second-BN partial sums")
        _direct_launch(A, B, out, stats, groups, _direct_geom(geo, dh, dw, tb, out, bias, addend, bwd, scales),
                       cfg[2] - DIRECT_BASE, bwd, shift)
        return
    C.conv_gemm(A, B, out, stats, bias, *geo, dh, dw, tb, groups, zero, addend, *bwd, *cfg, *scales, *xa3, shift,
                *xf2, mask, None, None, None, 0, **y2k)


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
# (512-channel 7x7: 266 vs 279 us); the others lost 1.3-2x (profiles/history/r6b_halo_probe_b1024.txt)
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


_PW_CFGS = None
PW_CONV = os.environ.get("IMGCLS_PW", "1") == "1"  # register-resident-weight 1x1 kernels (csrc/conv_pw.hip) as candidates
PW_FORCE = None  # tests: force a pointwise variant on every eligible launch
PW_COUNT = [0]   # pointwise-kernel launches (tests)
PW_BASE = 3000   # cfg[2] >= PW_BASE: the pointwise kernel, entry cfg - base


def conv_pw_cfgs():
    """The pointwise kernel's table: (output channels per block, k capacity)."""
    global _PW_CFGS
    if _PW_CFGS is None:
        _PW_CFGS = [tuple(c) for c in C.conv_pw_cfgs()]
    return _PW_CFGS


def _pw_ok(geo, dh, dw, tb, v=None):
    """A plain 1x1 stride-1 forward launch (csrc/conv_pw.hip::conv_pw_launch) that entry ``v`` covers: K fits
    its k capacity without a whole spare 32-wide chunk, and its channel tile is not wider than the layer."""
    m, co, k, ca, gh, gw, ih, iw, sa = geo[:9]
    if len(dh) != 1 or dh[0] or dw[0] or tb[0] or sa != 1 or (gh, gw) != (ih, iw) or k != ca or ca % 8 or co % 8:
        return False
    if geo[12] != 1 or geo[13] or geo[14] or (geo[10], geo[11]) != (gh, gw) or geo[15] % 4 or geo[16] % 4:
        return False
    if v is None:
        return True
    n_blk, k_cap = conv_pw_cfgs()[v]
    return k <= k_cap < k + 32 and n_blk < co + 16


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
DIRECT_CFGS = {0: (32, 32), 1: (32, 64), 2: (64, 32), 3: (64, 64), 4: (96, 32), 5: (64, 64)}
# variant 5: csrc/direct64.hip (weights resident in LDS, LDS-DMA double-buffered 8 x 32 patches) - exactly 64
# input channels and a 'same' 3x3 window (OH == H, OW == W): ResNet layer1 conv2 forward and data gradient


def _direct_variant_ok(v, dg) -> bool:
    cip, cot = DIRECT_CFGS[v]
    if dg[3] > cip or not (cot == 32 or dg[6] > 32):
        return False
    return v != 5 or (dg[3] == 64 and dg[4] == dg[1] and dg[5] == dg[2] and dg[6] % 8 == 0)


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
               xf=None, mask=None, y2=None):
    scratch = torch.empty_like(out)
    y2k = dict(bwd_y2=y2[0], bwd_coef2=y2[1], bwd_part2=torch.zeros_like(y2[2])) if y2 is not None else {}
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
                                                  addend, *bwd, *cfg, *scales, *xa3, None, *xf2, mask, None, None, None, 0, **y2k))
    if HALO_CONV and not fused and scales[0] is None:
        for v, (tm, bn, _wm, _wn, _bst, pmax) in enumerate(conv_halo_cfgs()):
            if v not in HALO_TUNE or not _halo_ok(geo, dh, dw, tm, pmax) or (bn > 64 and bn >= 2 * geo[1]) or \
                    (bn == 64 and geo[1] >= 256) or geo[0] < tm * 16:
                continue
            cfg = (0, 0, HALO_BASE + v)
            times[cfg] = _time_ms(lambda: C.conv_gemm(A, B, scratch, sst, bias, *geo, dh, dw, tb, groups, zero,
                                                      addend, *bwd, *cfg, *scales, *xa3, None, *xf2, mask, None, None, None, 0, **y2k))
    if DEEP_CONV and not fused and scales[0] is None and _deep_ok(geo, dh, dw):
        for v, (tm, bn, _wm, _wn, var) in enumerate(conv_deep_cfgs()):
            # var & 256 (32x32x16 MFMA blocks) is measured but not tuned: 5-10% slower than the same schedule on
            # 16x16x32 on every ResNet-50 shape (profiles/r10n_deep_mfma32_ab.txt)
            if var & (6 | 256) or (bn > 64 and bn >= 2 * geo[1]) or (bn == 64 and geo[1] >= 256) or geo[0] < tm * 8:
                continue
            cfg = (0, 0, DEEP_BASE + v)
            times[cfg] = _time_ms(lambda: C.conv_gemm(A, B, scratch, sst, bias, *geo, dh, dw, tb, groups, zero,
                                                      addend, *bwd, *cfg, *scales, *xa3, None, *xf2, mask, None, None, None, 0, **y2k))
    if PW_CONV and not fused and scales[0] is None and bias is None and addend is None and bwd[0] is None and \
            bwd[1] is None and mask is None and _pw_ok(geo, dh, dw, tb):
        for v in range(len(conv_pw_cfgs())):
            if _pw_ok(geo, dh, dw, tb, v):
                cfg = (0, 0, PW_BASE + v)
                times[cfg] = _time_ms(lambda: C.conv_gemm(A, B, scratch, sst, bias, *geo, dh, dw, tb, groups, zero,
                                                          addend, *bwd, *cfg, *scales, *xa3, None, *xf2, mask, None,
                                                          None, None, 0, **y2k))
    dg = _direct_geom(geo, dh, dw, tb, out, bias, addend, bwd, scales) if not fused and y2 is None else None
    if dg is not None:
        for v in DIRECT_CFGS:
            if _direct_variant_ok(v, dg):
                times[(0, 0, DIRECT_BASE + v)] = _time_ms(
                    lambda: _direct_launch(A, B, scratch, sst, groups, dg, v, bwd))
    TUNE_LOG.append((geo[0], geo[1], geo[2], times))
    return min(times, key=times.get)


def fp8_eligible(g: "ConvGeom") -> bool:
    return _shadows.FP8_FWD and g.Cx == g.Ci and g.Cx % 128 == 0 and g.Co % 8 == 0


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
# launches (ResNet-50 b1024 13344-13358 vs 13589-13626 img/s with only the 64-input form, profiles/history/r7n_*): off
FUSED_XA_BWD_N = os.environ.get("IMGCLS_FUSED_BWD_N", "0") == "1"
_CU_COUNT: dict = {}


def fused_bwd_eligible(g: ConvGeom, xa) -> bool:
    if not (FUSED_XA_BWD and xa is not None and g.kh == 1 and g.kw == 1 and g.sh == 1 and g.sw == 1
            and g.pt == 0 and g.pl == 0 and g.Cx == g.Ci and g.OH == g.H and g.OW == g.W):
        return False
    # 64 input channels and up to 256 outputs (layer1 conv3), or 64 outputs and 128 / 256 inputs (layer1 conv1)
    return (g.Ci == 64 and g.Co % 64 == 0 and g.Co <= 256) or (FUSED_XA_BWD_N and g.Co == 64 and g.Ci in (128, 256))


# The deferred downsample BN of a ResNet stage (``BwdLink.ds``: its output is only the residual of this BN) receives
# the same masked gradient dz as the residual BN: the data-gradient epilogue that produces dz also accumulates its
# (sum dz, sum dz * xhat_ds) - one read of y_ds there instead of a separate reduce pass over dz and y_ds.
DS_FUSE = os.environ.get("IMGCLS_DS_FUSE", "1") == "1"
DS_FUSE_COUNT = [0]


def _ds_partials(link, c, grp, dev, g):
    """(y_ds, coef_ds, part_ds) for the epilogue, or None (no deferred downsample BN on this link, no mask, or a
    data gradient whose pixels are remapped: the kernels carry the second partials on the direct map only)."""
    ds = getattr(link, "ds", None)
    if not DS_FUSE or ds is None or link.mask is None or ds.y is None or ds.done or ds.coef is None:
        return None
    if not (g.sh == 1 and g.sw == 1 and g.OH == g.H and g.OW == g.W):
        return None
    if ds.y.shape != link.y.shape or not ds.y.is_contiguous(memory_format=torch.channels_last):
        return None
    ds.part = ws(dev).take_part(c, grp)
    ds.groups = grp
    DS_FUSE_COUNT[0] += 1
    return ds.y, ds.coef, ds.part


def conv_fused_bwd_raw(dz, x, w_param, g: ConvGeom, xa, addend=None, link=None):
    """dX (as ``conv_dgrad_raw`` with ``xa``) and dW (into the parameter's arena slot or a fresh gradient
    buffer) of a ``fused_bwd_eligible`` conv from one launch; returns (dx, dw)."""
    dev = dz.device
    bwd = (None, None, None, None, 0, 1)
    mask = None
    y2 = None
    if link is not None:
        grp = stat_groups(g.N * g.H * g.W)
        link.part = ws(dev).take_part(g.Ci, grp)
        bwd = (link.y, link.res, link.coef, link.part, link.act, grp)
        mask = link.mask
        y2 = _ds_partials(link, g.Ci, grp, dev, g)
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
                xa[0], xa[1], None, None, None, 0, mask, x, wsp, dw.view(-1), blocks,
                **(dict(bwd_y2=y2[0], bwd_coef2=y2[1], bwd_part2=y2[2]) if y2 is not None else {}))
    if y2 is not None:
        link.ds.done = True
    FUSED_XA_BWD_COUNT[0] += 1
    return dx, dw


def conv_dgrad_raw(dy, w_param, g: ConvGeom, addend=None, link=None, xa=None, xa_out=None, wt=None):
    """dX = conv_transpose(dY, W) [+ addend], one MFMA GEMM per sub-pixel phase.

    With ``link`` (the producer BN of the conv input) the epilogue instead emits
    dz = act'(z) * dX and the producer's BN-backward partial sums (fused reduce).
    With ``xa`` = (y, coef) ``dy`` is the consuming BN's pre-elementwise gradient dz and the kernel
    forms dY = coef0*dz + coef1*y + coef2 on its A-operand loads (1x1 convs, ``XaLink``); with ``xa_out``
    (a tensor shaped like dy) the first column tile also stores that dY, so the weight gradient can read it
    plainly (``XA_OUT``).  ``wt``: the [Ci][T][Co] bf16 operand itself (concatenated siblings), else
    ``w_param``'s transposed shadow."""
    dev = dy.device
    bwd = (None, None, None, None, 0, 1)
    mask = None
    y2 = None
    if link is not None:
        grp = stat_groups(g.N * g.H * g.W)
        link.part = ws(dev).take_part(g.Ci, grp)
        bwd = (link.y, link.res, link.coef, link.part, link.act, grp)
        mask = link.mask
        y2 = _ds_partials(link, g.Ci, grp, dev, g)
    if wt is None:
        wt = weight_bf16_t(w_param, g.Co, g.T, g.Ci)
    dx = _empty_cl(g.N, g.Ci, g.H, g.W, dev)
    for ph, pw, gh, gw, dh, dw, tb in _dgrad_phases(g):
        if gh <= 0 or gw <= 0:
            continue
        geo = (g.N * gh * gw, g.Ci, len(tb) * g.Co, g.Co, gh, gw, g.OH, g.OW, 1, g.T * g.Co, g.H, g.W, g.sh,
               ph, pw, g.Ci, 0)
        _conv_gemm(dy, wt, dx, None, None, geo, dh, dw, tb, ws(dev).zero, addend, bwd,
                   xa=(xa if xa_out is None else (xa[0], xa[1], xa_out)) if (xa is not None and len(tb)) else None,
                   mask=mask, y2=y2)
    if y2 is not None:
        link.ds.done = True
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


WGRAD_DEEP = os.environ.get("IMGCLS_WGRAD_DEEP", "1") == "1"  # stages 13-15 (csrc/wgrad_deep.hip) as candidates
WGRAD_NARROW_TILES = os.environ.get("IMGCLS_WGRAD_NARROW_TILES", "1") == "1"  # stages 10-12 as tuner candidates
WGRAD_STAGES = int(os.environ.get("IMGCLS_WGRAD_STAGES", "0"))  # 0 = tuned with the split count; 1 | 2 | 3


WGRAD_WS = os.environ.get("IMGCLS_WGRAD_WS", "1") == "1"  # split-K partials: workspace slabs + reduce (0: atomics)
# ... except for layers of at most this many output pixels (N * OH * OW): there the split-K partials go straight into
# the zeroed gradient slot by fp32 atomics, which saves the reduce launch - the whole cost of a tiny layer's split
# (Inception-v3 b4 graph replay: ~75 wgrad_reduce launches of ~5 us in an 8.4 ms step).  Same box: Inception-v3 b4
# +3.7 % at this threshold; b32, b128 and ResNet-50 b64 unchanged; all-atomic weight gradients lose 3.5 % at b128 and
# an 8192-pixel threshold 2.2 % (its 8 x 8 layers), profiles/r15p_wgrad_atomic_small_layers_ab.txt
WGRAD_ATOMIC_PIX = int(os.environ.get("IMGCLS_WGRAD_ATOMIC_PIX", "6144"))
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
    if WGRAD_WS and splits > 1 and ntot % 8 == 0 and m > WGRAD_ATOMIC_PIX:
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
    if stages in (4, 7, 9, 13):
        return (-(-co // 256)) * (-(-ntot // 256))
    if stages == 16:  # 64 x 256 on 4 waves (Cout <= 64)
        return (-(-co // 64)) * (-(-ntot // 256))
    if stages in (14, 15):  # prefetch-depth-2 kernel (csrc/wgrad_deep.hip): 128 x 256 / 256 x 128
        return (-(-co // (128 if stages == 14 else 256))) * (-(-ntot // (256 if stages == 14 else 128)))
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
    if _common.DETERMINISTIC:  # one split: every dW element receives exactly one atomic contribution
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
        if WGRAD_DEEP and not (fx or ff):  # prefetch-depth-2 kernel, 4 waves of 128 x 128 / 64 x 128 / 128 x 64
            if g.Co >= 256 and ntot >= 256:
                cands += [(cand, 13) for cand in (256, 512, 768)]
            if g.Co >= 128 and ntot >= 256:
                cands += [(cand, 14) for cand in (256, 512, 768, 1024)]
            if g.Co >= 256 and ntot >= 128:
                cands += [(cand, 15) for cand in (256, 512, 768, 1024)]
        if g.Co <= 32:  # 32-row tiles: a 64-row tile would be half empty
            cands += [(cand, st) for st in (5, 6) for cand in blocks]
        if g.Co <= 64 and ntot >= 256:  # 64 x 256: one column tile where an XA / XF form re-forms per tile
            cands += [(cand, 16) for cand in blocks]
        if ntot <= 64 and WGRAD_NARROW_TILES:  # 64-column tiles: a 128-column tile is half empty (layer1 conv3)
            cands += [(cand, st) for st in (10, 11) for cand in blocks]
            if g.Co >= 256:
                cands += [(cand, 12) for cand in blocks if cand <= 1024]
        # (64 / 128 x 256 four-wave tiles, reading the narrow layers' dY half as often, were 5-70 % slower
        # on every ResNet-50 shape: profiles/history/r4d_wgrad_wide_tiles_probe.txt)
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


# names this part owns (ops/hip.py re-exports them)
_OWNED = (
    'CONV_FORCE_CFG', 'CONV_FORCE_FP8_CFG', 'CONV_STAGES', 'ConvGeom', 'DEEP_BASE', 'DEEP_CONV', 'DEEP_COUNT',
    'DEEP_FORCE', 'DIRECT_BASE', 'PW_BASE', 'PW_CONV', 'PW_COUNT', 'PW_FORCE', '_PW_CFGS', 'DIRECT_CFGS', 'DIRECT_CONV', 'DIRECT_DGRAD', 'DIRECT_FORCE', 'FUSED_XA_BWD',
    'FUSED_XA_BWD_COUNT', 'FUSED_XA_BWD_N', 'HALO_BASE', 'HALO_CONV', 'HALO_COUNT', 'HALO_FORCE', 'HALO_TUNE',
    'SKIP_WGRAD', 'TUNE_LOG', 'WGRAD_CANDIDATES', 'WGRAD_DEEP', 'WGRAD_MIN_K', 'WGRAD_NARROW_TILES', 'WGRAD_STAGES',
    'WGRAD_ATOMIC_PIX', 'WGRAD_TARGET_BLOCKS', 'WGRAD_TUNE_LOG', 'WGRAD_WS', '_CFGS', '_CU_COUNT', '_DEEP_CFGS', '_FP8_CFGS',
    '_HALO_CFGS', '_ORDER_IDX', '_STAGES_TUNED', '_WGRAD_TUNED', '_WGRAD_WS', '_conv_candidates',
    '_conv_forward_fp8', '_conv_gemm', '_deep_ok', '_dgrad_phases', '_direct_geom', '_direct_launch', '_direct_variant_ok', '_pw_ok', 'conv_pw_cfgs',
    '_fwd_taps', '_halo_ok', '_time_ms', '_tune_conv', '_weight_for_input', '_wgrad_config', '_wgrad_has',
    '_wgrad_launch', '_wgrad_plan', '_wgrad_split', '_wgrad_tiles', '_wgrad_ws', 'conv_cfgs', 'conv_deep_cfgs',
    'conv_dgrad_raw', 'conv_forward_raw', 'conv_fp8_cfgs', 'conv_fused_bwd_raw', 'conv_geom', 'conv_halo_cfgs',
    'fp8_eligible', 'fused_bwd_eligible', 'load_tuning', 'save_tuning', 'DS_FUSE', 'DS_FUSE_COUNT', '_ds_partials',
)
