"""Functional op layer the model zoo is written against.

Every model in ``models/`` expresses its forward pass with the handful of
primitives below (``conv_bn_act``, pooling, ``linear``, ``mlp``, ``se_gate``,
``drop_connect`` ...).  Each primitive has exactly two implementations:

* the **HIP path** (``ops/hip.py``): hand-written gfx950 kernels from
  ``csrc/*.hip`` operating on channels-last (NHWC) bf16 activations with fp32
  statistics/master weights.  Used for every CUDA (=HIP) tensor.
* the **reference path**: plain ATen ops in the module's own dtype.  Used on
  CPU (BASELINE config 1, the unit-test oracle) and, when explicitly requested
  with ``set_backend('torch')``, on the GPU to measure the reference stack
  (PyTorch DDP + SyncBatchNorm + MIOpen) on the same box.

This mirrors what the reference computes implicitly through torchvision /
efficientnet_pytorch modules (reference nn/classifier.py:11-37) but lets the
GPU path fuse conv -> BN -> (+residual) -> activation.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

_BACKEND = os.environ.get("IMGCLS_BACKEND", "auto")  # auto | hip | torch


def set_backend(name: str) -> None:
    global _BACKEND
    if name not in ("auto", "hip", "torch"):
        raise ValueError(f"unknown backend {name!r}")
    _BACKEND = name


def get_backend() -> str:
    return _BACKEND


def use_hip(x: torch.Tensor) -> bool:
    """HIP kernels run for every GPU tensor unless the torch backend is forced."""
    if not x.is_cuda:
        if _BACKEND == "hip":
            raise RuntimeError("backend 'hip' requested for a CPU tensor")
        return False
    return _BACKEND != "torch"


def _hip():
    from . import hip  # noqa: WPS433  (lazy: loads the native extension)
    return hip


# ---------------------------------------------------------------------------
# padding helpers
# ---------------------------------------------------------------------------
def conv_padding(conv, h: int, w: int):
    """Return (pad_top, pad_bottom, pad_left, pad_right) for ``conv``.

    ``conv.tf_same`` (set by the EfficientNet builder) selects TensorFlow
    "SAME" padding computed from the actual input size, as efficientnet_pytorch's
    Conv2dStaticSamePadding does for its configured image size.
    """
    kh, kw = conv.kernel_size
    sh, sw = conv.stride
    dh, dw = conv.dilation
    if getattr(conv, "tf_same", False):
        oh, ow = math.ceil(h / sh), math.ceil(w / sw)
        ph = max((oh - 1) * sh + (kh - 1) * dh + 1 - h, 0)
        pw = max((ow - 1) * sw + (kw - 1) * dw + 1 - w, 0)
        return ph // 2, ph - ph // 2, pw // 2, pw - pw // 2
    ph, pw = conv.padding
    return ph, ph, pw, pw


def _torch_conv(x, conv):
    pt, pb, pl, pr = conv_padding(conv, x.shape[-2], x.shape[-1])
    if (pt, pl) != (pb, pr):
        x = F.pad(x, (pl, pr, pt, pb))
        return F.conv2d(x, conv.weight, conv.bias, conv.stride, 0, conv.dilation, conv.groups)
    return F.conv2d(x, conv.weight, conv.bias, conv.stride, (pt, pl), conv.dilation, conv.groups)


def _act(x, act):
    if act is None:
        return x
    if act == "relu":
        return F.relu(x)
    if act == "silu":
        return F.silu(x)
    raise ValueError(act)


def _torch_bn(x, bn):
    sync = getattr(bn, "sync_group", None)
    if sync is not None and bn.training:
        from ..parallel.syncbn import sync_batch_norm
        return sync_batch_norm(x, bn, sync)
    return bn(x)


# ---------------------------------------------------------------------------
# primitives
# ---------------------------------------------------------------------------
def grad_slot(x, n: int = 2):
    """A gradient slot for a tensor with exactly ``n`` consumers that each take ``slot=`` (HIP path;
    None otherwise): their backward contributions are summed inside the consumers' own kernels."""
    if use_hip(x) and x.requires_grad and torch.is_grad_enabled():
        return _hip().GradSlot(n)
    return None


def conv_bn_act(x, conv, bn, act="relu", residual=None, x_slot=None, res_slot=None, exclusive_input=False,
                out=None, pool=None, prepool=None, defer_act=False, defer_res=False):
    """act(bn(conv(x)) [+ residual]).

    Reference equivalents: torchvision ``BasicConv2d`` (conv -> BN -> ReLU),
    ResNet ``Bottleneck``/``BasicBlock`` tails (BN -> +identity -> ReLU) and
    efficientnet_pytorch ``MBConvBlock`` (conv -> BN -> swish).
    ``pool`` = (kernel, stride, padding): a max pool follows the activation (the ResNet / Inception
    stems); the HIP path fuses it into the BN passes.
    ``prepool`` = (kernel, stride, padding): an average pool (count_include_pad) precedes the conv (the
    Inception ``branch_pool``); for a 1x1 conv the HIP path runs the conv first and pools its narrower
    output - both are linear, so conv1x1(avgpool(x)) == avgpool(conv1x1(x)).
    ``defer_act``: the caller feeds the result only to the next ``conv_bn_act`` (as its exclusive input);
    the HIP path may then skip writing act(bn(y)) and let that conv apply the BN on its operand loads.
    ``defer_res``: the result (no activation) is used only as the ``residual`` of one later ``conv_bn_act``
    (a ResNet downsample branch); the HIP path then skips writing bn(y) and that BN applies it on its loads.
    """
    if prepool is not None:
        if residual is not None or pool is not None:
            raise ValueError("conv_bn_act(prepool=...) takes a plain avgpool -> conv -> BN -> act")
        if use_hip(x):
            return _hip().pool_conv_bn_act(x, conv, bn, act, prepool, x_slot,
                                           (out[0].hip(), out[1]) if (out is not None and _hip().CONCAT_INPLACE)
                                           else None, out)
        x = F.avg_pool2d(x, *prepool)
    if pool is not None:  # stem: max_pool2d(act(bn(conv(x))), *pool) - kernel, stride, padding
        if residual is not None or x_slot is not None or out is not None:
            raise ValueError("conv_bn_act(pool=...) takes a plain conv -> BN -> act")
        if use_hip(x):
            return _hip().conv_bn_act_pool(x, conv, bn, act, pool, exclusive_input)
        return F.max_pool2d(_act(_torch_bn(_torch_conv(x, conv), bn), act), *pool)
    if use_hip(x):
        hout = (out[0].hip(), out[1]) if (out is not None and _hip().CONCAT_INPLACE) else None
        return _hip().conv_bn_act(x, conv, bn, act, residual, x_slot, res_slot, exclusive_input, hout,
                                  defer_act=defer_act, defer_res=defer_res)
    y = _torch_bn(_torch_conv(x, conv), bn)
    if residual is not None:
        y = y + residual
    return _act(y, act)


def siblings_ok(x, pairs) -> bool:
    """The HIP path can run these (conv, bn) pairs - 1x1 convs of the same ``x`` - as one GEMM
    (``conv_bn_act_siblings``); the caller then gives ``x`` one gradient-slot consumer for all of them."""
    return use_hip(x) and _hip().siblings_eligible(x, pairs)


def conv_bn_act_siblings(x, pairs, outs, act="relu", x_slot=None):
    """[act(bn(conv(x))) for (conv, bn) in pairs] as one concatenated-output GEMM (HIP path, ``siblings_ok``);
    ``outs[i]`` = (ConcatPlan, branch) writes that result into the concat output in place."""
    h = _hip()
    hout = [(o[0].hip(), o[1]) if (o is not None and h.CONCAT_INPLACE) else None for o in outs]
    res = h.conv_bn_act_siblings(x, pairs, hout, act, x_slot)
    return res


def conv(x, conv_mod):
    """Plain convolution (with optional bias), no normalisation."""
    if use_hip(x):
        return _hip().conv(x, conv_mod)
    return _torch_conv(x, conv_mod)


def max_pool2d(x, kernel_size, stride, padding=0, slot=None):
    if use_hip(x):
        return _hip().max_pool2d(x, kernel_size, stride, padding, slot)
    return F.max_pool2d(x, kernel_size, stride, padding)


def avg_pool2d(x, kernel_size, stride, padding=0, slot=None):
    """count_include_pad=True semantics (torch default, used by torchvision Inception)."""
    if use_hip(x):
        return _hip().avg_pool2d(x, kernel_size, stride, padding, slot)
    return F.avg_pool2d(x, kernel_size, stride, padding)


def global_avg_pool(x):
    """adaptive_avg_pool2d(x, 1) + flatten -> [N, C]."""
    if use_hip(x):
        return _hip().global_avg_pool(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


def linear(x, lin, act=None):
    if use_hip(x):
        return _hip().linear(x, lin, act)
    return _act(F.linear(x, lin.weight, lin.bias), act)


def mlp(x, seq):
    """The reference classifier head: Linear/ReLU stack (nn/classifier.py:26-34)."""
    if use_hip(x):
        return _hip().mlp(x, seq)
    return seq(x)


def dropout(x, p, training):
    if p == 0.0 or not training:
        return x
    if use_hip(x):
        return _hip().dropout(x, p)
    return F.dropout(x, p, True)


class ConcatPlan:
    """A channel concat whose branches write their outputs in place: pass ``out=(plan, i)`` to the
    branch's final ``conv_bn_act`` and ``buf=plan`` to ``cat_channels`` (HIP path: ``hip.ConcatBuffer``;
    the reference path ignores the plan and concatenates with ``torch.cat``)."""

    def __init__(self, channels):
        self.channels = list(channels)
        self._hip = None

    def hip(self):
        if self._hip is None:
            self._hip = _hip().ConcatBuffer(self.channels)
        return self._hip


def concat_buffer(channels) -> ConcatPlan:
    return ConcatPlan(channels)


def cat_channels(xs, buf=None):
    if use_hip(xs[0]):
        h = _hip()
        return h.cat_channels(xs, buf.hip() if (buf is not None and h.CONCAT_INPLACE) else None)
    return torch.cat(xs, 1)


def add(x, y):
    if use_hip(x):
        return _hip().add(x, y)
    return x + y


def se_gate(x, se_reduce, se_expand, exclusive_input=False):
    """Squeeze-and-excitation: x * sigmoid(expand(swish(reduce(avgpool(x))))).  ``exclusive_input``: the gate
    is x's only consumer (HIP path: its backward runs the backward reduce of the BN that produced x)."""
    if use_hip(x):
        return _hip().se_gate(x, se_reduce, se_expand, exclusive_input)
    s = F.adaptive_avg_pool2d(x, 1)
    s = se_expand(F.silu(se_reduce(s)))
    return torch.sigmoid(s) * x


def drop_connect(x, p, training):
    """efficientnet_pytorch utils.drop_connect: per-sample stochastic depth."""
    if not training or p == 0.0:
        return x
    if use_hip(x):
        return _hip().drop_connect(x, p)
    keep = 1.0 - p
    mask = torch.floor(keep + torch.rand([x.shape[0], 1, 1, 1], dtype=x.dtype, device=x.device))
    return x / keep * mask


def cross_entropy(logits, labels, weight=None):
    """CrossEntropyLoss(weight) with mean reduction: sum_i w_yi*nll_i / sum_i w_yi
    (reference train.py:157-158)."""
    if use_hip(logits):
        return _hip().cross_entropy(logits, labels, weight)
    return F.cross_entropy(logits.float(), labels, weight=weight)


def prepare_input(x, stem=None):
    """Move/convert a batch to the layout the active path expects.

    HIP path: channels-last bf16 (NHWC in memory); with ``stem`` (a 7x7 stride-2 first conv) the
    fp32 batch may be left for the space-to-depth stem to convert.  Reference path: unchanged.
    """
    if use_hip(x):
        return _hip().prepare_input(x, stem=stem)
    return x
