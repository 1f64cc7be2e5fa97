"""Classifier head, loss, input preparation, concat / add / dropout / drop-connect and the
squeeze-excitation gate.

Split out of ``ops/hip.py`` (the facade that re-exports every name here).
"""
from __future__ import annotations

import os

import torch

from ..grad_arena import grad_buffer
from . import common as _common
from .common import BF16, C, CL, _cl, _empty_cl, ws
from .convbn import _syncbn_bwd_start, stem_s2d_eligible


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
                      exclusive_input and _common.FUSE_BN_BWD and SE_LINK)


# names this part owns (ops/hip.py re-exports them)
_OWNED = (
    'AddFn', 'CONCAT_INPLACE', 'CatFn', 'ConcatBuffer', 'CrossEntropyFn', 'DropoutFn', 'MlpFn', 'SEFn',
    'SE_FUSED', 'SE_LINK', 'ScaleRowsFn', '_AFFINE_CACHE', '_mm', 'add', 'cat_channels', 'cross_entropy',
    'drop_connect', 'dropout', 'linear', 'mlp', 'prepare_input', 'se_gate',
)
