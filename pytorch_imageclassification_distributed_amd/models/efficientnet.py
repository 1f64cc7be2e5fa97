"""EfficientNet-B0..B7 (efficientnet_pytorch topology and parameter names).

Reference: ``EfficientNet.from_pretrained('efficientnet-b3')`` (reference
nn/classifier.py:17-18).  ``efficientnet_pytorch`` is not installed here, so the
network is re-declared with the same module tree (``_conv_stem, _bn0,
_blocks.{i}.{_expand_conv,_bn0,_depthwise_conv,_bn1,_se_reduce,_se_expand,
_project_conv,_bn2}, _conv_head, _bn1, _fc``), TF "SAME" padding, swish,
squeeze-excitation, drop-connect (stochastic depth) and dropout.  BN uses
momentum 0.01 / eps 1e-3 as efficientnet_pytorch's defaults.

The head attribute is ``_fc`` (reference defect A5: the reference assigns
``encoder.fc`` and crashes; ``Classifier`` here targets ``_fc``).
"""
from __future__ import annotations

import math
import re
from collections import namedtuple

import torch.nn as nn

from ..ops import functional as Fx

BlockArgs = namedtuple("BlockArgs", ["num_repeat", "kernel_size", "stride", "expand_ratio",
                                     "input_filters", "output_filters", "se_ratio", "id_skip"])

_B0_BLOCKS = [
    "r1_k3_s11_e1_i32_o16_se0.25", "r2_k3_s22_e6_i16_o24_se0.25",
    "r2_k5_s22_e6_i24_o40_se0.25", "r3_k3_s22_e6_i40_o80_se0.25",
    "r3_k5_s11_e6_i80_o112_se0.25", "r4_k5_s22_e6_i112_o192_se0.25",
    "r1_k3_s11_e6_i192_o320_se0.25",
]

# name: (width, depth, resolution, dropout)
EFFICIENTNET_PARAMS = {
    "efficientnet-b0": (1.0, 1.0, 224, 0.2), "efficientnet-b1": (1.0, 1.1, 240, 0.2),
    "efficientnet-b2": (1.1, 1.2, 260, 0.3), "efficientnet-b3": (1.2, 1.4, 300, 0.3),
    "efficientnet-b4": (1.4, 1.8, 380, 0.4), "efficientnet-b5": (1.6, 2.2, 456, 0.4),
    "efficientnet-b6": (1.8, 2.6, 528, 0.5), "efficientnet-b7": (2.0, 3.1, 600, 0.5),
}


def _decode(s: str) -> BlockArgs:
    opts = {}
    for part in s.split("_"):
        m = re.split(r"(\d.*)", part)
        if len(m) >= 2:
            opts[m[0]] = m[1]
    return BlockArgs(int(opts["r"]), int(opts["k"]), int(opts["s"][0]), int(opts["e"]),
                     int(opts["i"]), int(opts["o"]), float(opts["se"]) if "se" in opts else None,
                     "noskip" not in s)


def round_filters(filters, width, divisor=8, min_depth=None):
    if not width:
        return filters
    filters *= width
    min_depth = min_depth or divisor
    new = max(min_depth, int(filters + divisor / 2) // divisor * divisor)
    if new < 0.9 * filters:
        new += divisor
    return int(new)


def round_repeats(repeats, depth):
    return int(math.ceil(depth * repeats)) if depth else repeats


def _conv(cin, cout, k, stride=1, groups=1, bias=False):
    c = nn.Conv2d(cin, cout, k, stride, 0, groups=groups, bias=bias)
    c.tf_same = True  # TF "SAME" padding (Conv2dStaticSamePadding)
    return c


class MBConvBlock(nn.Module):
    def __init__(self, args: BlockArgs, bn_mom=0.01, bn_eps=1e-3):
        super().__init__()
        self._block_args = args
        self.has_se = args.se_ratio is not None and 0 < args.se_ratio <= 1
        self.id_skip = args.id_skip
        inp = args.input_filters
        oup = inp * args.expand_ratio
        if args.expand_ratio != 1:
            self._expand_conv = _conv(inp, oup, 1)
            self._bn0 = nn.BatchNorm2d(oup, momentum=bn_mom, eps=bn_eps)
        self._depthwise_conv = _conv(oup, oup, args.kernel_size, args.stride, groups=oup)
        self._bn1 = nn.BatchNorm2d(oup, momentum=bn_mom, eps=bn_eps)
        if self.has_se:
            nsq = max(1, int(inp * args.se_ratio))
            self._se_reduce = _conv(oup, nsq, 1, bias=True)
            self._se_expand = _conv(nsq, oup, 1, bias=True)
        self._project_conv = _conv(oup, args.output_filters, 1)
        self._bn2 = nn.BatchNorm2d(args.output_filters, momentum=bn_mom, eps=bn_eps)

    def forward(self, inputs, drop_connect_rate=None):
        a = self._block_args
        x = inputs
        skip = self.id_skip and a.stride == 1 and a.input_filters == a.output_filters
        # exclusive_input: the conv is the tensor's only consumer, so (HIP path) its data-gradient kernel
        # can run the backward reduce of the BN that produced the tensor (the block input feeds the skip
        # connection too when ``skip``)
        if a.expand_ratio != 1:
            x = Fx.conv_bn_act(x, self._expand_conv, self._bn0, "silu", exclusive_input=not skip)
        x = Fx.conv_bn_act(x, self._depthwise_conv, self._bn1, "silu",
                           exclusive_input=a.expand_ratio != 1 or not skip)
        if self.has_se:
            x = Fx.se_gate(x, self._se_reduce, self._se_expand, exclusive_input=True)
        if skip and not (drop_connect_rate and self.training):
            return Fx.conv_bn_act(x, self._project_conv, self._bn2, None, residual=inputs)
        x = Fx.conv_bn_act(x, self._project_conv, self._bn2, None)
        if skip:
            x = Fx.drop_connect(x, drop_connect_rate, self.training)
            x = Fx.add(x, inputs)
        return x


class EfficientNet(nn.Module):
    def __init__(self, width, depth, dropout, num_classes=1000, drop_connect_rate=0.2,
                 blocks=_B0_BLOCKS):
        super().__init__()
        bn_mom, bn_eps = 0.01, 1e-3
        self.drop_connect_rate = drop_connect_rate
        out = round_filters(32, width)
        self._conv_stem = _conv(3, out, 3, 2)
        self._bn0 = nn.BatchNorm2d(out, momentum=bn_mom, eps=bn_eps)
        self._blocks = nn.ModuleList()
        args = None
        for s in blocks:
            args = _decode(s)
            args = args._replace(input_filters=round_filters(args.input_filters, width),
                                 output_filters=round_filters(args.output_filters, width),
                                 num_repeat=round_repeats(args.num_repeat, depth))
            self._blocks.append(MBConvBlock(args, bn_mom, bn_eps))
            if args.num_repeat > 1:
                args = args._replace(input_filters=args.output_filters, stride=1)
            for _ in range(args.num_repeat - 1):
                self._blocks.append(MBConvBlock(args, bn_mom, bn_eps))
        cin = args.output_filters
        out = round_filters(1280, width)
        self._conv_head = _conv(cin, out, 1)
        self._bn1 = nn.BatchNorm2d(out, momentum=bn_mom, eps=bn_eps)
        self._avg_pooling = nn.AdaptiveAvgPool2d(1)
        self._dropout = nn.Dropout(dropout)
        self._fc = nn.Linear(out, num_classes)

    def extract_features(self, x):
        x = Fx.conv_bn_act(x, self._conv_stem, self._bn0, "silu")
        n = len(self._blocks)
        for idx, block in enumerate(self._blocks):
            dcr = self.drop_connect_rate * float(idx) / n if self.drop_connect_rate else None
            x = block(x, drop_connect_rate=dcr)
        return Fx.conv_bn_act(x, self._conv_head, self._bn1, "silu")

    def input_spec(self):
        """(space-to-depth stem input, per-channel scale, shift) (ops/hip.py input_from_u8)."""
        return (False, None, None)

    def forward(self, x):
        x = Fx.prepare_input(x)
        x = Fx.global_avg_pool(self.extract_features(x))
        x = Fx.dropout(x, self._dropout.p, self.training)
        return Fx.mlp(x, self._fc) if isinstance(self._fc, nn.Sequential) else Fx.linear(x, self._fc)


def efficientnet(name: str, num_classes=1000):
    w, d, _res, p = EFFICIENTNET_PARAMS[name]
    return EfficientNet(w, d, p, num_classes=num_classes)


def efficientnet_b0(num_classes=1000):
    return efficientnet("efficientnet-b0", num_classes)


def efficientnet_b3(num_classes=1000):
    return efficientnet("efficientnet-b3", num_classes)
