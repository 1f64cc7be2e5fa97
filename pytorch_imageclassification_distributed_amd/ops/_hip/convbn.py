"""Conv / BatchNorm autograd Functions: gradient slots, SyncBN backward start, the fused BN-backward (XA)
and BN-apply (XF) links, ConvFn, the space-to-depth stem, depthwise, dense and bias convs, BN + act
(+ residual, + pool) and the ``conv_bn_act`` entry points.

Split out of ``ops/hip.py`` (the facade that re-exports every name here).
"""
from __future__ import annotations

import os

import torch

from ...parallel.peer import (PeerWork, peer_channel, stats_all_reduce_,
                               stats_all_reduce_async, side_stream as peer_side_stream)
from ..grad_arena import arena_slot, grad_buffer
from . import common as _common
from . import shadows as _shadows
from . import gemm as _gemm
from .common import ACT, BF16, C, CL, SHIFT_STATS, _cl, _empty_cl, _sync_group, stat_groups, stat_shift, ws
from .shadows import FP8, ensure_channels_last_weight, weight_bf16, weight_bf16_t
from .gemm import (ConvGeom, _wgrad_plan, conv_dgrad_raw, conv_forward_raw, conv_fused_bwd_raw, conv_geom,
                   fused_bwd_eligible)
from .streams import _on_side, conv_wgrad_raw
from .pool import AvgPoolFn, _pool_args, avg_pool2d, channel_slice_stride, max_pool2d


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
        if torch.cuda.is_current_stream_capturing():
            # a HIP-graph capture keeps it on the capturing stream (a forked capture replays slowly on this
            # runtime); same channel, same call order on every rank
            pc.comm.bn_bwd(link.part, link.part_rows(), c, link.count_t, dgamma, dbeta, k)
            link.pending = (None, None, dgamma, dbeta, k)
            SYNCBN_EARLY_COUNT[0] += 1
            return
        side = peer_side_stream(dev)
        side.wait_stream(cur)
        from ...parallel import comm_timer
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
                 "groups", "count_t", "ds")

    def __init__(self):
        self.y = self.coef = self.res = self.mask = self.part = None
        self.ds = None  # the deferred downsample BN's link when this BN's residual is its output (gemm.DS_FUSE)
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
# XA with the dY written once by the data gradient (its first column tile stores the dY it formed in LDS):
# the weight gradient then reads dY plainly instead of re-forming it from dz and y in every column tile
# (the fused wgrads ran VALU-bound at 10-20 % MFMA busy).  Same bytes (one dY write on the
# compute stream against one fewer tensor read on the side stream), no replicated transform.
# ResNet-50 b1024, same box, 2 rounds each: 13904 / 13942 img/s without, 14240 / 14221 with (profiles/r12b_xa_out_ab.txt)
XA_OUT = os.environ.get("IMGCLS_XA_OUT", "1") == "1"
XA_OUT_COUNT = [0]


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


def _xa_out_ok(g) -> bool:
    """Every dY element passes through the data gradient's A operand exactly once in a tile of the first
    column: a 1x1 conv without padding (stride 1, or the single non-empty phase of stride 2)."""
    return g.kh == 1 and g.kw == 1 and g.pt == 0 and g.pl == 0 and g.Cx == g.Ci


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
# Off by default: measured on ResNet-50 b1024 (profiles/history/r5f_fusion_ab.txt) it does not pay - the bn_apply passes
# it removes are small (the non-residual ones were 3.5 ms of the 77 ms step) and a 3x3 consumer re-applies the
# map once per tap
FUSE_XF = os.environ.get("IMGCLS_BN_XF", "0") == "1"
XF_COUNT = [0]  # convs that read a deferred BN output (tests / diagnostics)


class XfHold:
    """The deferred BN output's map: ``coef`` = the BN's [scale | shift | mean | invstd] (written by its
    forward), ``act`` = 0 (identity) or 1 (ReLU).  Rides on the BN's output tensor as ``_imgcls_xf``; that
    tensor holds y (the BN input), so only a conv taking the map (``ConvFn``) or ``XfMaterializeFn`` may
    read it."""

    __slots__ = ("coef", "act", "link")

    def __init__(self):
        self.coef = None
        self.act = 0
        self.link = None  # a deferred residual: the deferred BN's backward link


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
            and not _shadows.FP8_FWD and not dense_conv_eligible(x, conv))


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
                if xa is not None and XA_OUT and ctx.needs_input_grad[1] and _xa_out_ok(g):
                    xo = torch.empty_like(dy)
                    dx = conv_dgrad_raw(dy, w, g, addend=addend, link=link, xa=xa, xa_out=xo)
                    dy, xa = xo, None  # the weight gradient reads the materialised dY
                    XA_OUT_COUNT[0] += 1
                else:
                    dx = conv_dgrad_raw(dy, w, g, addend=addend, link=link, xa=xa)
            if link is not None:
                link.done = True
                if link.group is not None:
                    # SyncBN: start the producer BN's backward all-reduce now, so its latency overlaps
                    # this conv's weight gradient instead of sitting between two dependent kernels
                    _syncbn_bwd_start(link)
                ds = link.ds
                if ds is not None and ds.done and ds.group is not None:
                    _syncbn_bwd_start(ds)  # (the deferred downsample BN's partials came from the same epilogue)
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
    The result carries a marker so prepare_input / the stem pass it through unchanged.  Odd image sizes
    take the NHWC8 form even for an s2d stem (the stem then runs as a plain 7x7 implicit GEMM), and the
    NHWC8 kernel handles any pixel count (299 x 299 maps, partial last batches)."""
    s2d, sc, sh = spec
    n, h, w, _ = u8.shape
    a = [1.0 / (255.0 * std[c]) for c in range(3)]
    b = [-mean[c] / std[c] for c in range(3)]
    if sc is not None:
        a = [a[c] * sc[c] for c in range(3)]
        b = [b[c] * sc[c] + sh[c] for c in range(3)]
    if s2d and h % 2 == 0 and w % 2 == 0:
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
    def forward(ctx, x, w, conv, want_stats, shift=None, s2d_hw=None, xa=None):
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
        ctx.xa = xa
        ctx.save_for_backward(xs, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        xs, w = ctx.saved_tensors
        g = ctx.g
        # STEM_XA: the pooled BN's backward handed over dz and its map; the weight gradient forms dY on its loads
        xa = ctx.xa.take(dy) if ctx.xa is not None else None
        dy = _cl(dy)
        dw = None
        if ctx.needs_input_grad[1]:
            m, ntot = g.N * g.OH * g.OW, g.T * g.Cx
            kps, splits, stages = _wgrad_plan(g, dy, xs, m, ntot, xa=xa)
            full = torch.zeros(g.Co * ntot, dtype=torch.float32, device=dy.device)
            idx = _s2d_index(dy.device)
            slot = arena_slot(w)
            dw = slot if slot is not None else grad_buffer(w, zero=False)

            # the last weight gradient of backward: on the compute stream (idle by then) it runs beside the
            # side stream's backlog instead of behind it (conv_wgrad_raw, padded-channel path)
            _gemm._wgrad_launch(dy, xs, full, g, m, ntot, kps, splits, stages, xa=xa)
            dw.permute(0, 2, 3, 1).reshape(g.Co, 147).copy_(full.view(g.Co, ntot)[:, idx])
        return None, dw, None, None, None, None, None


# ---------------------------------------------------------------------------
# depthwise convolution (EfficientNet)
# ---------------------------------------------------------------------------
# The depthwise forward also produces the consumer BN's batch statistics (csrc/dwconv.hip dw_fwd_rs_kernel EPI 2),
# as the GEMM convs' epilogues do: the BN's separate statistics pass over y disappears (IMGCLS_DW_STATS=0: keep it)
DW_STATS = os.environ.get("IMGCLS_DW_STATS", "1") == "1"
DW_STATS_COUNT = [0]  # depthwise launches that produced their BN's statistics (tests / diagnostics)


def dw_stats_eligible(x, conv) -> bool:
    # (deterministic mode keeps the BN's own statistics pass: its rows take one contribution each)
    if not DW_STATS or _common.DETERMINISTIC:
        return False
    g = conv_geom(x, conv)
    return C.dw_fwd_stats_ok(g.N, g.Co, g.OH, g.OW, g.kh, g.kw, g.sh, g.sw)


class DwConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, conv, fuse_bwd=False, want_stats=False, shift=None):
        g = conv_geom(x, conv)
        wt = weight_bf16_t(w, g.Co, g.T, 1)
        y = _empty_cl(g.N, g.Co, g.OH, g.OW, x.device)
        if want_stats:
            grp = stat_groups(g.N * g.OH * g.OW)  # the rows the BN reduces (_bn_coef)
            stats = ws(x.device).stats_buf(g.Co, grp)
            C.dw_fwd(x, wt, y, stats, g.N, g.H, g.W, g.Co, g.OH, g.OW, g.kh, g.kw, g.sh, g.sw, g.pt, g.pl,
                     G=grp, shift=shift)
            DW_STATS_COUNT[0] += 1
        else:
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
                if _common.DETERMINISTIC:  # one partial row per block: every address gets one contribution
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
        return dx, dw, None, None, None, None


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
            from ...parallel import comm_timer
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
    from ...parallel import comm_timer
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


# Training BN of a small tensor (<= IMGCLS_BN_FIN_MAX elements): the partial-row reduce and finalize run inside the
# apply kernel (csrc/bn.hip bn_fin_apply_kernel) - one launch instead of two, which is what a BN costs at the
# reference's Inception-v3 b4 launch (graph replay, ~5 us per kernel)
BN_FIN = os.environ.get("IMGCLS_BN_FIN", "1") == "1"
BN_FIN_MAX = int(os.environ.get("IMGCLS_BN_FIN_MAX", str(1 << 21)))
BN_FIN_COUNT = [0]
# the backward counterpart (bn_reduce_bwd inside bn_bwd_elemt, csrc/bn.hip bn_fin_bwd_kernel).  Its first form (one
# dependent row load per iteration) measured no better than the two launches (profiles/r15v_bn_fin_bwd_ab.txt); with
# two rows of loads in flight per lane: Inception-v3 b4 +1 %, b32 +1 %, ResNet-50 b64 unchanged (profiles/r16a_*)
BN_FIN_BWD = os.environ.get("IMGCLS_BN_FIN_BWD", "1") == "1"
BN_FIN_BWD_COUNT = [0]  # BN backwards whose reduce rode in the elementwise pass

# The residual BN's ReLU mask (1 bit per element, written by bn_apply) replaces the consumer dgrad epilogue's
# re-read of the residual when it recomputes z = bn(y) + res > 0: ~11 GB less per ResNet-50 b1024 step.
RELU_MASK = os.environ.get("IMGCLS_RELU_MASK", "1") == "1"


class BNActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, gamma, beta, res, bn, act, stats_ready, res_slot=None, link=None, cat=None, xa=None,
                shift=None, defer=None, res_hold=None):
        dev = y.device
        n, c, h, w = y.shape
        rows = n * h * w
        a = ACT[act]
        fin = (BN_FIN and bn.training and res is None and res_hold is None and defer is None and a <= 2
               and c % 8 == 0 and c <= 64 * 64 and rows * c <= BN_FIN_MAX and not _shadows.FP8_FWD
               and not _common.DETERMINISTIC and _sync_group(bn) is None)
        if fin:
            # small tensor: the finalize rides in the apply (one launch instead of two)
            coef, group, count_t = torch.empty(4 * c, dtype=torch.float32, device=dev), None, None
            grp = stat_groups(rows)
            part = ws(dev).stats_buf(c, grp)
            if not stats_ready:
                C.bn_stats(y, rows, c, part, grp, shift=shift)
            mom = bn.momentum if bn.momentum is not None else 0.1
            track = bn.track_running_stats and bn.running_mean is not None
            rs = (bn.running_mean, bn.running_var, bn.num_batches_tracked) if track else (None, None, None)
            if cat is not None:
                cbuf, idx = cat
                dst, ldo, off = cbuf.ensure(n, h, w, dev), cbuf.total, cbuf.offs[idx]
                out = cbuf.part(idx, c)
            else:
                out = dst = _empty_cl(n, c, h, w, dev)
                ldo, off = c, 0
            C.bn_fin_apply(y, part, grp, float(rows), gamma, beta, *rs, mom, bn.eps, coef, shift, dst, rows, c, ldo,
                           off, a, ws(dev).fin_ctr)
            BN_FIN_COUNT[0] += 1
        else:
            coef, group, count_t = _bn_coef(y, gamma, beta, bn, stats_ready, shift)
        # res_hold: the residual is a deferred BN output (it holds that BN's input); this apply forms it
        res_coef = None
        if res_hold is not None:
            if res_hold.act != 0:
                raise RuntimeError("deferred residual BN: identity activation only")
            will_mask = bn.training and link is not None  # (the mask condition of the plain apply below)
            if (cat is not None or defer is not None or a != 1 or _shadows.FP8_FWD or not RELU_MASK
                    or not C.bn_res_coef_ok(will_mask)):
                # any other form materializes the residual first (what the deferred BN would have written); the
                # fused form needs the ReLU mask, which the backward consumers read instead of the residual, and
                # the flat apply walk (bn_res_coef_ok: the A/B knobs IMGCLS_BN_WALK / unroll can turn it off)
                r = _empty_cl(n, c, h, w, dev)
                C.bn_apply(res, res_hold.coef, None, r, rows, c, c, 0, 0)
                res, res_hold = r, None
            else:
                res_coef = res_hold.coef
                RES_DEFER_COUNT[0] += 1
        if fin:
            pass  # (applied above)
        elif defer is not None:
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
        elif _shadows.FP8_FWD and c % 128 == 0:  # the consuming conv reads an MX-FP8 copy: produce it here
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
            C.bn_apply(y, coef, res, out, rows, c, c, 0, a, mask=mask, res_coef=res_coef)
            if link is not None:
                link.mask = mask
        ctx.act, ctx.group, ctx.rows, ctx.c = a, group, rows, c
        ctx.training = bn.training
        ctx.count_t = count_t
        ctx.res_slot = res_slot
        ctx.link = None
        if link is not None and bn.training:  # (grad mode is always off inside forward)
            # (a deferred residual holds the downsample BN's input: the consuming conv's epilogue reads the mask
            # instead, and consumers that cannot take a residual still see one and decline the link)
            link.y, link.coef, link.res, link.act = y, coef, res, a
            link.group, link.params, link.c, link.rows = group, (gamma, beta), c, rows
            link.count_t = count_t
            # a deferred downsample residual: the epilogue that produces this BN's dz also takes that BN's partials
            link.ds = res_hold.link if (res_coef is not None and res_slot is None) else None
            ctx.link = link
        ctx.has_res = res is not None
        ctx.res_coef = res_coef
        ctx.params = (gamma, beta)
        ctx.xa = xa if bn.training else None
        ctx.save_for_backward(y, coef, res if res is not None else y)
        return out

    @staticmethod
    def backward(ctx, gout):  # (with ``defer`` too: gout is the gradient w.r.t. act(bn(y)))
        y, coef, res = ctx.saved_tensors
        res = res if ctx.has_res else None
        if res is not None and ctx.res_coef is not None and not (ctx.link is not None and ctx.link.done):
            # the activation is recomputed from z = bn(y) + residual below: form the deferred residual
            n_, c_, h_, w_ = res.shape
            r = _empty_cl(n_, c_, h_, w_, res.device)
            C.bn_apply(res, ctx.res_coef, None, r, n_ * h_ * w_, c_, c_, 0, 0)
            res = r
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
            _common.FUSED_BWD_COUNT[0] += 1
            pending = link.pending
            link.y = link.coef = link.res = link.mask = link.part = link.pending = link.params = link.count_t = None
            link.ds = None
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
        fin = (BN_FIN_BWD and xa is None and pending is None and ctx.training and ctx.group is None and c % 8 == 0
               and rows * c <= BN_FIN_MAX and not _common.DETERMINISTIC)
        if fin:  # small tensor: the partial-row reduce rides in the elementwise pass (one launch instead of two)
            dgamma = grad_buffer(ctx.params[0], zero=False)
            dbeta = grad_buffer(ctx.params[1], zero=False)
            dy = torch.empty_like(y, memory_format=CL)
            C.bn_fin_bwd(part, grp, float(rows), dgamma, dbeta, None if dz is not None else g, y, coef, res, dz, dy,
                         rows, c, ctx.act, 0 if dz is not None else ldg, ws(dev).fin_ctr)
            BN_FIN_BWD_COUNT[0] += 1
        elif pending is not None:  # SyncBN all-reduce launched early by the consuming conv's backward
            sums, work, dgamma, dbeta, k = pending
            if work is not None:  # (None: ran on this stream, inside a graph capture)
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
        elif not fin:
            dy = torch.empty_like(y, memory_format=CL)
            C.bn_bwd_elemt(None if dz is not None else g, y, coef, k, res, dz, dy, rows, c, ctx.act,
                           0 if dz is not None else ldg)
        dres = dz if ctx.has_res else None
        if dres is not None and ctx.res_slot is not None:
            dres = ctx.res_slot.deliver(dres)
        return dy, dgamma, dbeta, dres, None, None, None, None, None, None, None, None, None, None


class BNActPoolFn(torch.autograd.Function):
    """maxpool(act(BN(y))) for network stems (ResNet conv1 -> bn1 -> relu -> maxpool 3/2/1, Inception
    Conv2d_2b / Conv2d_4a -> maxpool 3/2/0).  The forward pools straight from ``y`` (the
    full-resolution activation is never written or re-read).  The backward is maxpool_bwd -> BN backward:
    gathering the pooled gradient inside both BN-backward passes measured slower (docs/DESIGN.md)."""

    @staticmethod
    def forward(ctx, y, gamma, beta, bn, act, stats_ready, pool, shift=None, xa=None):
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
        # STEM_XA: the ReLU mask comes from the pooled output in the pool backward, and the producer conv's
        # weight gradient forms dY itself (XaLink) - no bn_bwd_elemt pass, no dY tensor
        ctx.xa = xa if (xa is not None and bn.training and a == ACT["relu"] and
                        C.maxpool_bwd_relu_ok(n, h, w, c, *geo[4:])) else None
        ctx.save_for_backward(y, coef, idx, out if ctx.xa is not None else y)
        return out

    @staticmethod
    def backward(ctx, gout):
        y, coef, idx, out = ctx.saved_tensors
        dev = y.device
        n, c, h, w = y.shape
        rows = n * h * w
        _, _, oh, ow, kh, kw, sh, sw, ph, pw = ctx.geo
        xa = ctx.xa
        g = _empty_cl(n, c, h, w, dev)
        grp = stat_groups(rows)
        part = ws(dev).stats_buf(c, grp)
        # POOL_BN_REDUCE: the pool backward also takes the BN-backward partial sums of the dz it writes
        red = xa is not None and POOL_BN_REDUCE and C.maxpool_bwd_reduce_ok(n, h, w, c, kh, kw, sh, sw, ph, pw)
        C.maxpool_bwd(_cl(gout), idx, g, n, h, w, c, oh, ow, kh, kw, sh, sw, ph, pw,
                      relu_out=out if xa is not None else None,
                      **(dict(bn_y=y, bn_coef=coef, part=part, G=grp) if red else {}))
        act = 0 if xa is not None else ctx.act  # (g is already dz: masked by the pooled output)
        if red:
            POOL_BN_REDUCE_COUNT[0] += 1
        else:
            C.bn_bwd_reduce(g, y, coef, None, None, rows, c, act, part, grp)
        xac = torch.empty(3 * c, dtype=torch.float32, device=dev) if xa is not None else None
        k, dgamma, dbeta = _bn_bwd_k(part, grp, c, rows, ctx.training, ctx.group, ctx.count_t, ctx.params, dev,
                                     coef=coef, xa=xac)
        if xa is not None:
            xa.dz, xa.y, xa.coef = g, y, xac
            STEM_XA_COUNT[0] += 1
            return g, dgamma, dbeta, None, None, None, None, None, None
        dy = torch.empty_like(y, memory_format=CL)
        C.bn_bwd_elemt(g, y, coef, k, None, None, dy, rows, c, act)
        return dy, dgamma, dbeta, None, None, None, None, None, None


STEM_POOL_FUSE = os.environ.get("IMGCLS_STEM_POOL_FUSE", "1") == "1"
# The ResNet stem's BN backward hands its dz and elementwise map to the stem conv's weight gradient (XA), which is
# the only consumer of the stem's dY: the bn_bwd_elemt pass over the 112 x 112 x 64 activation and its dY tensor
# disappear from the tail of every step (IMGCLS_STEM_XA=0: keep them)
STEM_XA = os.environ.get("IMGCLS_STEM_XA", "1") == "1"
STEM_XA_COUNT = [0]
# with STEM_XA the stem's max-pool backward also accumulates the BN-backward partial sums of the dz it writes (one
# read of y there instead of a separate reduce pass re-reading dz and y; IMGCLS_POOL_BN_REDUCE=0: the separate pass)
POOL_BN_REDUCE = os.environ.get("IMGCLS_POOL_BN_REDUCE", "1") == "1"
POOL_BN_REDUCE_COUNT = [0]


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
        xa = XaLink() if (STEM_XA and bn.training and torch.is_grad_enabled() and conv.weight.requires_grad) else None
        y = StemS2dFn.apply(x, conv.weight, conv, bn.training, shift, getattr(x, "_imgcls_s2d", None), xa)
        return BNActPoolFn.apply(y, bn.weight, bn.bias, bn, act, bn.training, (k, s, p), shift, xa)
    if conv.groups != 1 or conv.bias is not None:
        raise NotImplementedError("conv_bn_act_pool: grouped conv / conv bias")
    y = ConvFn.apply(_cl(x), conv.weight, conv, bn.training, None, exclusive_input and _common.FUSE_BN_BWD, None, shift)
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
        from ..functional import conv_bn_act as _f_conv_bn_act
        return _f_conv_bn_act(avg_pool2d(x, *prepool, slot=x_slot), conv, bn, act, out=out_plan)
    x = _cl(x)
    ensure_channels_last_weight(conv)
    y = ConvFn.apply(x, conv.weight, conv, False, x_slot, False)
    yp = AvgPoolFn.apply(y, k, s, p, None)
    return BNActFn.apply(yp, bn.weight, bn.bias, None, bn, act, False, None, None, out, None, stat_shift(bn))


# A ResNet downsample BN (no activation) whose output is only the residual of its block's last BN is not
# applied at all: it hands that BN its input y and coefficients (XfHold), and the residual BN's apply forms
# sc3 * y3 + sh3 + (sc_ds * y_ds + sh_ds) itself - one read + one write of the downsample output fewer per
# stage (the four bn_apply passes were 1.04 ms of the ResNet-50 b1024 step, profiles/r13a_step_breakdown.txt)
RES_DEFER = os.environ.get("IMGCLS_RES_DEFER", "1") == "1"
RES_DEFER_COUNT = [0]  # residual BNs that applied a deferred downsample BN (tests / diagnostics)


def conv_bn_act(x, conv, bn, act, residual, x_slot=None, res_slot=None, exclusive_input=False, out=None,
                defer_act=False, defer_res=False):
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
        link = BwdLink() if (_common.FUSE_BN_BWD and bn.training and torch.is_grad_enabled()) else None
        out = BNActFn.apply(y, bn.weight, bn.bias, None, bn, act, bn.training, None, link, None, None, shift)
        if link is not None:
            out._imgcls_link = link
        return out
    x = _cl(x)
    res_hold = getattr(residual, "_imgcls_xf", None) if residual is not None else None
    if residual is not None:
        residual = _cl(residual)
    ensure_channels_last_weight(conv)
    depthwise = conv.groups > 1
    dense = False
    xa = None
    if depthwise:
        if not (conv.groups == conv.in_channels == conv.out_channels):
            raise NotImplementedError("grouped (non-depthwise) convolution")
        ready = bn.training and dw_stats_eligible(x, conv)
        y = DwConvFn.apply(x, conv.weight, conv, exclusive_input and _common.FUSE_BN_BWD and DW_LINK, ready,
                           shift if ready else None)
    elif dense_conv_eligible(x, conv) and x.shape[2] * x.shape[3] > 1:
        dense = True
        y = DenseConvFn.apply(x, conv.weight, conv, bn.training, shift)
        ready = bn.training
    else:
        if conv.groups != 1:
            raise NotImplementedError("grouped convolution")
        xa = XaLink() if (bn.training and torch.is_grad_enabled() and xa_eligible(x, conv)) else None
        y = ConvFn.apply(x, conv.weight, conv, bn.training, x_slot, exclusive_input and _common.FUSE_BN_BWD, xa, shift, xf)
        xf = None
        ready = bn.training
    if xf is not None:
        raise RuntimeError("deferred BN output reached a consumer without the fused map")
    if conv.bias is not None:
        raise NotImplementedError("conv bias before BatchNorm")
    link = BwdLink() if (_common.FUSE_BN_BWD and bn.training and torch.is_grad_enabled()) else None
    hold = XfHold() if (((defer_act and FUSE_XF and ACT[act] <= 1) or (defer_res and RES_DEFER and ACT[act] == 0))
                        and bn.training and torch.is_grad_enabled() and residual is None
                        and out is None and not _shadows.FP8_FWD) else None
    res_out = BNActFn.apply(y, bn.weight, bn.bias, residual, bn, act, ready, res_slot, link, out,
                            xa if not depthwise and not dense else None, shift, hold, res_hold)
    if link is not None:
        res_out._imgcls_link = link
    if hold is not None:
        if defer_res:
            hold.link = link
        res_out._imgcls_xf = hold
    return res_out


# Sibling 1x1 convs sharing one input (Inception's branch heads: InceptionA 64 + 48 + 64, InceptionC 192 + c7 + c7,
# InceptionE 320 + 384 + 448) as ONE implicit GEMM with their output channels concatenated: x is read once by the
# forward and by the weight gradient, and the data gradient is one K = sum(Co) GEMM.  That replaces three gradient-slot
# accumulations.  Each branch's BN then normalises its channel slice in place with the one-launch BN kernels (row
# strides: csrc/bn.hip bn_fin_apply_kernel / bn_fin_bwd_kernel), writing its output where that branch wrote it
# (a concat slice or its own tensor).  Per block and step this is 2 + 2 x 2 fewer GEMM launches, which is what a
# step costs at the reference's Inception-v3 b4 launch.  The merged path gives up the per-branch fusions (XA,
# consumer-epilogue BN reduces) and still wins at every batch measured: b4 +3.5 %, b32 +3.1 %, b256 +2-4 %, b512 +3.9 %
# (profiles/r16q_*); IMGCLS_SIBLINGS_MAX caps the concatenated output's elements, IMGCLS_SIBLINGS=0 turns it off.
SIBLINGS = os.environ.get("IMGCLS_SIBLINGS", "1") == "1"
SIBLINGS_MAX = int(os.environ.get("IMGCLS_SIBLINGS_MAX", str(1 << 30)))
SIBLINGS_COUNT = [0]


def siblings_eligible(x, pairs) -> bool:
    """Every (conv, bn) is a plain 1x1 stride-1 conv of ``x`` followed by a training BN without SyncBN, and the
    concatenated output is small enough for the one-launch BN kernels."""
    if (not SIBLINGS or _common.DETERMINISTIC or _shadows.FP8_FWD or not torch.is_grad_enabled() or x.dim() != 4
            or x.shape[1] % 8 or getattr(x, "_imgcls_xf", None) is not None):
        return False
    co = 0
    for conv, bn in pairs:
        if not (bn.training and conv.groups == 1 and conv.bias is None and tuple(conv.kernel_size) == (1, 1)
                and tuple(conv.stride) == (1, 1) and tuple(conv.padding) == (0, 0) and tuple(conv.dilation) == (1, 1)
                and not getattr(conv, "tf_same", False) and conv.in_channels == x.shape[1]
                and conv.out_channels % 8 == 0 and bn.num_features == conv.out_channels
                and bn.track_running_stats and bn.running_mean is not None and _sync_group(bn) is None):
            return False
        co += conv.out_channels
    n, _, h, w = x.shape
    return co <= 64 * 64 and n * h * w * co <= SIBLINGS_MAX


def _sibling_geom(x, convs) -> ConvGeom:
    """The 1x1 geometry of the merged GEMM: the first sibling's, with the concatenated output channels."""
    g0 = conv_geom(x, convs[0])
    co = sum(c.out_channels for c in convs)
    cache = convs[0].__dict__.setdefault("_imgcls_sib_geom", {})
    g = cache.get((x.shape, co))
    if g is None:
        g = ConvGeom.__new__(ConvGeom)
        for k in ConvGeom.__slots__:
            setattr(g, k, getattr(g0, k))
        g.Co = co
        cache[(x.shape, co)] = g
    return g


class SiblingConvFn(torch.autograd.Function):
    """y = x conv [W_0; W_1; ...] (1x1) with the BN statistics of every output channel in the GEMM epilogue."""

    @staticmethod
    def forward(ctx, x, slot, convs, shift, *weights):
        g = _sibling_geom(x, convs)
        wb = torch.cat([weight_bf16(w) for w in weights])  # [sum Co][Ci]
        stats = ws(x.device).stats_buf(g.Co, stat_groups(g.N * g.OH * g.OW))
        y = conv_forward_raw(x, None, g, stats=stats, wb=wb, shift=shift)
        ctx.g, ctx.slot = g, slot
        ctx.save_for_backward(x, *weights)
        SIBLINGS_COUNT[0] += 1
        return y

    @staticmethod
    def backward(ctx, dy):
        x, *weights = ctx.saved_tensors
        g = ctx.g
        dy = _cl(dy)
        dx = None
        if ctx.needs_input_grad[0]:
            wt = torch.cat([weight_bf16_t(w, w.shape[0], 1, g.Ci).view(g.Ci, w.shape[0]) for w in weights], dim=1)
            slot = ctx.slot
            addend = slot.t if slot is not None else None  # (the other consumers' sum rides in as the addend)
            dx = conv_dgrad_raw(dy, None, g, addend=addend, wt=wt.contiguous())
            if slot is not None:
                dx = slot.deliver(dx, fused=addend is not None)
        dws = [None] * len(weights)
        if any(ctx.needs_input_grad[4:]):
            m, ntot = g.N * g.OH * g.OW, g.T * g.Cx
            kps, splits, stages = _wgrad_plan(g, dy, x, m, ntot)
            for i, w in enumerate(weights):
                if ctx.needs_input_grad[4 + i]:
                    dws[i] = grad_buffer(w, zero=False)

            def launch():  # the merged weight gradient, then its split into the siblings' gradient slots
                full = torch.zeros(g.Co * ntot, dtype=torch.float32, device=dy.device)  # (small splits add atomically)
                _gemm._wgrad_launch(dy, x, full, g, m, ntot, kps, splits, stages)
                off = 0
                for w, d in zip(weights, dws):
                    if d is not None:
                        d.copy_(full[off:off + w.numel()].view(w.shape[0], w.shape[1], 1, 1))
                    off += w.numel()
            # on the weight-gradient side stream, as every other conv's (joined when backward ends)
            _on_side(dy.device, launch, dy, x, *[d for d in dws if d is not None])
        return (dx, None, None, None, *dws)


class SiblingBNFn(torch.autograd.Function):
    """act_i(bn_i(y[:, slice_i])) for every sibling: one launch per BN in each direction, reading its channel slice
    of the merged GEMM output in place (row stride sum(Co)); outputs go to a concat slice or their own tensor."""

    @staticmethod
    def forward(ctx, y, bns, acts, outs, shifted, *params):
        dev = y.device
        n, ctot, h, w = y.shape
        rows = n * h * w
        grp = stat_groups(rows)
        part = ws(dev).stats_buf(ctot, grp)
        results, coefs, off = [], [], 0
        for i, bn in enumerate(bns):
            c = bn.num_features
            coef = torch.empty(4 * c, dtype=torch.float32, device=dev)
            mom = bn.momentum if bn.momentum is not None else 0.1
            if outs[i] is not None:
                cbuf, idx = outs[i]
                dst, ldo, c_off = cbuf.ensure(n, h, w, dev), cbuf.total, cbuf.offs[idx]
                out = cbuf.part(idx, c)
            else:
                out = dst = _empty_cl(n, c, h, w, dev)
                ldo, c_off = c, 0
            C.bn_fin_apply(y[:, off:off + c], part[off:], grp, float(rows), params[2 * i], params[2 * i + 1],
                           bn.running_mean, bn.running_var, bn.num_batches_tracked, mom, bn.eps, coef,
                           bn.running_mean if shifted else None, dst, rows, c, ldo, c_off, ACT[acts[i]],
                           ws(dev).fin_ctr, ldy=ctot, ldp=ctot)
            results.append(out)
            coefs.append(coef)
            off += c
        ctx.bns, ctx.acts = bns, acts
        ctx.params = params
        ctx.save_for_backward(y, *coefs)
        return tuple(results)

    @staticmethod
    def backward(ctx, *gouts):
        y, *coefs = ctx.saved_tensors
        dev = y.device
        n, ctot, h, w = y.shape
        rows = n * h * w
        grp = stat_groups(rows)
        dy = _empty_cl(n, ctot, h, w, dev)
        grads, off = [], 0
        for i, bn in enumerate(ctx.bns):
            c = bn.num_features
            gout = gouts[i]
            if gout is None:
                gout = torch.zeros((n, c, h, w), dtype=y.dtype, device=dev).contiguous(memory_format=CL)
            ldg = channel_slice_stride(gout)  # a concat's gradient arrives as a channel slice: read in place
            g = gout if ldg else _cl(gout)
            a = ACT[ctx.acts[i]]
            part = ws(dev).take_part(c, grp)
            C.bn_bwd_reduce(g, y[:, off:off + c], coefs[i], None, None, rows, c, a, part, grp, ldg, ldy=ctot)
            dgamma = grad_buffer(ctx.params[2 * i], zero=False)
            dbeta = grad_buffer(ctx.params[2 * i + 1], zero=False)
            C.bn_fin_bwd(part, grp, float(rows), dgamma, dbeta, g, y[:, off:off + c], coefs[i], None, None,
                         dy[:, off:off + c], rows, c, a, ldg, ws(dev).fin_ctr, ldy=ctot, ldd=ctot)
            ws(dev).give_part(part)
            grads += [dgamma, dbeta]
            off += c
        return (dy, None, None, None, None, *grads)


def conv_bn_act_siblings(x, pairs, outs, act="relu", x_slot=None):
    """[act(bn_i(conv_i(x)))] for sibling 1x1 convs of one input (``siblings_eligible``), as one GEMM; ``outs[i]`` =
    (ConcatBuffer, branch) or None; ``x_slot``: x's gradient slot (this call is ONE consumer of it)."""
    x = _cl(x)
    convs = [c for c, _ in pairs]
    bns = [b for _, b in pairs]
    for c in convs:
        ensure_channels_last_weight(c)
    shifts = [stat_shift(b) for b in bns]  # (each BN's statistics pivot; the GEMM epilogue sums about their concat)
    shifted = all(t is not None for t in shifts)
    y = SiblingConvFn.apply(x, x_slot, convs, torch.cat(shifts) if shifted else None, *[c.weight for c in convs])
    params = [t for b in bns for t in (b.weight, b.bias)]
    return list(SiblingBNFn.apply(y, bns, [act] * len(bns), list(outs), shifted, *params))


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


# depthwise dgrad runs its producer BN's backward reduce: measured 0.6 % slower on EfficientNet-B0 (the extra
# y loads and coefficients lift the row-strip kernels to 2 waves per SIMD), so opt-in
DW_LINK = os.environ.get("IMGCLS_DW_LINK", "0") == "1"


# names this part owns (ops/hip.py re-exports them)
_OWNED = (
    'BNActFn', 'BNActPoolFn', 'BN_FIN', 'BN_FIN_BWD', 'BN_FIN_BWD_COUNT', 'BN_FIN_COUNT', 'BN_FIN_MAX', 'BwdLink', 'ConvBiasFn', 'ConvFn', 'DW_LINK', 'DW_STATS', 'DW_STATS_COUNT',
    'DenseConvFn', 'DwConvFn', 'dw_stats_eligible',
    'FUSE_XA', 'FUSE_XF', 'GradSlot', 'PEER_BN_MAX_C', 'POOL_CONV_SWAP', 'RELU_MASK', 'RES_DEFER', 'RES_DEFER_COUNT',
    'STEM_DIRECT',
    'POOL_BN_REDUCE', 'POOL_BN_REDUCE_COUNT', 'STEM_POOL_FUSE', 'STEM_S2D', 'STEM_XA', 'STEM_XA_COUNT', 'SYNCBN_EARLY_COUNT', 'StemS2dFn', 'XA_COUNT', 'XA_MAX_REP', 'XA_NARROW_OFF',
    'XF_COUNT', 'XF_MAX_REP', 'XA_OUT', 'XA_OUT_COUNT', '_xa_out_ok', 'XaLink', 'XfHold', 'XfMaterializeFn', '_S2D_INDEX', '_as_pixel_rows',
    '_bn_bwd_k', '_bn_coef', '_dense_geom', '_rep', '_s2d_geom', '_s2d_index', '_syncbn_bwd_start', 'conv',
    'conv_bn_act', 'conv_bn_act_pool', 'dense_conv_eligible', 'input_from_u8', 'materialize_deferred',
    'pool_conv_bn_act', 'stem_s2d_conv', 'stem_s2d_eligible', 'xa_eligible', 'xf_eligible',
    'SIBLINGS', 'SIBLINGS_COUNT', 'SIBLINGS_MAX', 'SiblingBNFn', 'SiblingConvFn', '_sibling_geom', 'conv_bn_act_siblings',
    'siblings_eligible',
)
