"""Inception-v3 (torchvision topology and parameter names, incl. the AuxLogits head).

Reference: ``models.inception_v3(pretrained=True)`` with ``AuxLogits.fc``
replaced by ``Linear(768, num_classes)`` (reference nn/classifier.py:20-23); the
training loop consumes ``(logits, aux_logits)`` in train mode and ``logits`` in
eval mode (reference train.py:48-56, 87).

Every ``BasicConv2d`` is conv(bias=False) -> BN(eps=1e-3) -> ReLU, which the GPU
path runs as one fused HIP conv->BN->ReLU unit.  ``transform_input`` (torchvision
enables it only together with ImageNet weights) is folded into the input
conversion kernel.
"""
from __future__ import annotations

from collections import namedtuple

import torch
import torch.nn as nn

from ..ops import functional as Fx

InceptionOutputs = namedtuple("InceptionOutputs", ["logits", "aux_logits"])


class BasicConv2d(nn.Module):
    def __init__(self, cin, cout, **kw):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, bias=False, **kw)
        self.bn = nn.BatchNorm2d(cout, eps=0.001)

    def forward(self, x, exclusive=False, slot=None, out=None, pool=None, prepool=None, defer=False):
        """``exclusive``: this conv is the only consumer of ``x`` (a chain-internal conv), which lets its
        dgrad epilogue run the producer's BN-backward reduce; ``slot``: x feeds exactly two convs;
        ``out``: (concat plan, branch) - write the result into the block's concat output in place;
        ``pool``: (kernel, stride, padding) of a max pool applied to the result (stem); ``prepool``: of an
        average pool applied to ``x`` first (``branch_pool``); ``defer``: the result feeds only the next
        conv of the chain (the HIP path lets that conv apply this BN + ReLU on its operand loads)."""
        return Fx.conv_bn_act(x, self.conv, self.bn, "relu", x_slot=slot, exclusive_input=exclusive, out=out,
                              pool=pool, prepool=prepool, defer_act=defer)


def _pairs(mods):
    """(conv, bn) of BasicConv2d modules (the sibling 1x1 heads of an Inception block)."""
    return [(m.conv, m.bn) for m in mods]


class InceptionA(nn.Module):
    def __init__(self, cin, pool_features):
        super().__init__()
        self.branch1x1 = BasicConv2d(cin, 64, kernel_size=1)
        self.branch5x5_1 = BasicConv2d(cin, 48, kernel_size=1)
        self.branch5x5_2 = BasicConv2d(48, 64, kernel_size=5, padding=2)
        self.branch3x3dbl_1 = BasicConv2d(cin, 64, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, kernel_size=3, padding=1)
        self.branch_pool = BasicConv2d(cin, pool_features, kernel_size=1)

    def forward(self, x):
        cat = Fx.concat_buffer([64, 64, 96, self.branch_pool.conv.out_channels])  # branches write in place
        heads = [self.branch1x1, self.branch5x5_1, self.branch3x3dbl_1]
        if Fx.siblings_ok(x, _pairs(heads)):  # the three 1x1 heads as one GEMM (HIP path, small steps)
            s = Fx.grad_slot(x, 2)
            b1, t5, t3 = Fx.conv_bn_act_siblings(x, _pairs(heads), [(cat, 0), None, None], x_slot=s)
        else:
            s = Fx.grad_slot(x, 4)  # x feeds three convs and the pool: summed inside their backward kernels
            b1 = self.branch1x1(x, slot=s, out=(cat, 0))
            t5 = self.branch5x5_1(x, slot=s)
            t3 = self.branch3x3dbl_1(x, slot=s, defer=True)
        b5 = self.branch5x5_2(t5, True, out=(cat, 1))
        b3 = self.branch3x3dbl_3(self.branch3x3dbl_2(t3, True), True, out=(cat, 2))
        bp = self.branch_pool(x, slot=s, prepool=(3, 1, 1), out=(cat, 3))
        return Fx.cat_channels([b1, b5, b3, bp], cat)


class InceptionB(nn.Module):
    def __init__(self, cin):
        super().__init__()
        self.branch3x3 = BasicConv2d(cin, 384, kernel_size=3, stride=2)
        self.branch3x3dbl_1 = BasicConv2d(cin, 64, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(64, 96, kernel_size=3, padding=1)
        self.branch3x3dbl_3 = BasicConv2d(96, 96, kernel_size=3, stride=2)

    def forward(self, x):
        s = Fx.grad_slot(x, 3)
        cat = Fx.concat_buffer([384, 96, x.shape[1]])  # the pool branch is copied in
        b3 = self.branch3x3(x, slot=s, out=(cat, 0))
        bd = self.branch3x3dbl_3(self.branch3x3dbl_2(self.branch3x3dbl_1(x, slot=s, defer=True), True), True,
                                 out=(cat, 1))
        bp = Fx.max_pool2d(x, 3, 2, 0, slot=s)
        return Fx.cat_channels([b3, bd, bp], cat)


class InceptionC(nn.Module):
    def __init__(self, cin, channels_7x7):
        super().__init__()
        c7 = channels_7x7
        self.branch1x1 = BasicConv2d(cin, 192, kernel_size=1)
        self.branch7x7_1 = BasicConv2d(cin, c7, kernel_size=1)
        self.branch7x7_2 = BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7_3 = BasicConv2d(c7, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_1 = BasicConv2d(cin, c7, kernel_size=1)
        self.branch7x7dbl_2 = BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_3 = BasicConv2d(c7, c7, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7dbl_4 = BasicConv2d(c7, c7, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7dbl_5 = BasicConv2d(c7, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch_pool = BasicConv2d(cin, 192, kernel_size=1)

    def forward(self, x):
        cat = Fx.concat_buffer([192, 192, 192, 192])
        heads = [self.branch1x1, self.branch7x7_1, self.branch7x7dbl_1]
        if Fx.siblings_ok(x, _pairs(heads)):  # the three 1x1 heads as one GEMM (HIP path, small steps)
            s = Fx.grad_slot(x, 2)
            b1, b7, bd = Fx.conv_bn_act_siblings(x, _pairs(heads), [(cat, 0), None, None], x_slot=s)
        else:
            s = Fx.grad_slot(x, 4)
            b1 = self.branch1x1(x, slot=s, out=(cat, 0))
            # chain-internal outputs are deferred (their consumer applies BN + ReLU; c7 = 160 materialises them)
            b7 = self.branch7x7_1(x, slot=s, defer=True)
            bd = self.branch7x7dbl_1(x, slot=s, defer=True)
        b7 = self.branch7x7_3(self.branch7x7_2(b7, True, defer=True), True, out=(cat, 1))
        bd = self.branch7x7dbl_3(self.branch7x7dbl_2(bd, True, defer=True), True, defer=True)
        bd = self.branch7x7dbl_5(self.branch7x7dbl_4(bd, True, defer=True), True, out=(cat, 2))
        bp = self.branch_pool(x, slot=s, prepool=(3, 1, 1), out=(cat, 3))
        return Fx.cat_channels([b1, b7, bd, bp], cat)


class InceptionD(nn.Module):
    def __init__(self, cin):
        super().__init__()
        self.branch3x3_1 = BasicConv2d(cin, 192, kernel_size=1)
        self.branch3x3_2 = BasicConv2d(192, 320, kernel_size=3, stride=2)
        self.branch7x7x3_1 = BasicConv2d(cin, 192, kernel_size=1)
        self.branch7x7x3_2 = BasicConv2d(192, 192, kernel_size=(1, 7), padding=(0, 3))
        self.branch7x7x3_3 = BasicConv2d(192, 192, kernel_size=(7, 1), padding=(3, 0))
        self.branch7x7x3_4 = BasicConv2d(192, 192, kernel_size=3, stride=2)

    def forward(self, x):
        cat = Fx.concat_buffer([320, 192, x.shape[1]])
        heads = [self.branch3x3_1, self.branch7x7x3_1]
        if Fx.siblings_ok(x, _pairs(heads)):  # the two 1x1 heads as one GEMM (HIP path)
            s = Fx.grad_slot(x, 2)
            t3, t7 = Fx.conv_bn_act_siblings(x, _pairs(heads), [None, None], x_slot=s)
        else:
            s = Fx.grad_slot(x, 3)
            t3 = self.branch3x3_1(x, slot=s, defer=True)
            t7 = self.branch7x7x3_1(x, slot=s, defer=True)
        b3 = self.branch3x3_2(t3, True, out=(cat, 0))
        b7 = self.branch7x7x3_2(t7, True, defer=True)
        b7 = self.branch7x7x3_4(self.branch7x7x3_3(b7, True, defer=True), True, out=(cat, 1))
        bp = Fx.max_pool2d(x, 3, 2, 0, slot=s)
        return Fx.cat_channels([b3, b7, bp], cat)


class InceptionE(nn.Module):
    def __init__(self, cin):
        super().__init__()
        self.branch1x1 = BasicConv2d(cin, 320, kernel_size=1)
        self.branch3x3_1 = BasicConv2d(cin, 384, kernel_size=1)
        self.branch3x3_2a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3_2b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch3x3dbl_1 = BasicConv2d(cin, 448, kernel_size=1)
        self.branch3x3dbl_2 = BasicConv2d(448, 384, kernel_size=3, padding=1)
        self.branch3x3dbl_3a = BasicConv2d(384, 384, kernel_size=(1, 3), padding=(0, 1))
        self.branch3x3dbl_3b = BasicConv2d(384, 384, kernel_size=(3, 1), padding=(1, 0))
        self.branch_pool = BasicConv2d(cin, 192, kernel_size=1)

    def forward(self, x):
        cat = Fx.concat_buffer([320, 384, 384, 384, 384, 192])
        heads = [self.branch1x1, self.branch3x3_1, self.branch3x3dbl_1]
        if Fx.siblings_ok(x, _pairs(heads)):  # the three 1x1 heads as one GEMM (HIP path, small steps)
            s = Fx.grad_slot(x, 2)
            b1, b3, td = Fx.conv_bn_act_siblings(x, _pairs(heads), [(cat, 0), None, None], x_slot=s)
        else:
            s = Fx.grad_slot(x, 4)
            b1 = self.branch1x1(x, slot=s, out=(cat, 0))
            b3 = self.branch3x3_1(x, slot=s)
            td = self.branch3x3dbl_1(x, slot=s, defer=True)
        s3 = Fx.grad_slot(b3)  # b3 and bd each feed exactly two convs: paired gradient slots
        b3a, b3b = self.branch3x3_2a(b3, slot=s3, out=(cat, 1)), self.branch3x3_2b(b3, slot=s3, out=(cat, 2))
        bd = self.branch3x3dbl_2(td, True)
        sd = Fx.grad_slot(bd)
        bda, bdb = self.branch3x3dbl_3a(bd, slot=sd, out=(cat, 3)), self.branch3x3dbl_3b(bd, slot=sd, out=(cat, 4))
        bp = self.branch_pool(x, slot=s, prepool=(3, 1, 1), out=(cat, 5))
        return Fx.cat_channels([b1, b3a, b3b, bda, bdb, bp], cat)


class InceptionAux(nn.Module):
    def __init__(self, cin, num_classes):
        super().__init__()
        self.conv0 = BasicConv2d(cin, 128, kernel_size=1)
        self.conv1 = BasicConv2d(128, 768, kernel_size=5)
        self.conv1.stddev = 0.01
        self.fc = nn.Linear(768, num_classes)
        self.fc.stddev = 0.001

    def forward(self, x):
        x = Fx.avg_pool2d(x, 5, 3, 0)
        x = self.conv1(self.conv0(x), True)
        x = Fx.global_avg_pool(x)
        return Fx.mlp(x, self.fc) if isinstance(self.fc, nn.Sequential) else Fx.linear(x, self.fc)


class Inception3(nn.Module):
    def __init__(self, num_classes=1000, aux_logits=True, transform_input=False, dropout=0.5):
        super().__init__()
        self.aux_logits = aux_logits
        self.transform_input = transform_input
        self.Conv2d_1a_3x3 = BasicConv2d(3, 32, kernel_size=3, stride=2)
        self.Conv2d_2a_3x3 = BasicConv2d(32, 32, kernel_size=3)
        self.Conv2d_2b_3x3 = BasicConv2d(32, 64, kernel_size=3, padding=1)
        self.maxpool1 = nn.MaxPool2d(kernel_size=3, stride=2)
        self.Conv2d_3b_1x1 = BasicConv2d(64, 80, kernel_size=1)
        self.Conv2d_4a_3x3 = BasicConv2d(80, 192, kernel_size=3)
        self.maxpool2 = nn.MaxPool2d(kernel_size=3, stride=2)
        self.Mixed_5b = InceptionA(192, pool_features=32)
        self.Mixed_5c = InceptionA(256, pool_features=64)
        self.Mixed_5d = InceptionA(288, pool_features=64)
        self.Mixed_6a = InceptionB(288)
        self.Mixed_6b = InceptionC(768, channels_7x7=128)
        self.Mixed_6c = InceptionC(768, channels_7x7=160)
        self.Mixed_6d = InceptionC(768, channels_7x7=160)
        self.Mixed_6e = InceptionC(768, channels_7x7=192)
        self.AuxLogits = InceptionAux(768, num_classes) if aux_logits else None
        self.Mixed_7a = InceptionD(768)
        self.Mixed_7b = InceptionE(1280)
        self.Mixed_7c = InceptionE(2048)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.dropout = nn.Dropout(p=dropout)
        self.fc = nn.Linear(2048, num_classes)
        for m in self.modules():  # torchvision init
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                std = float(getattr(m, "stddev", 0.1))
                nn.init.trunc_normal_(m.weight, mean=0.0, std=std, a=-2, b=2)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    # (x - mean_imagenet)/std_imagenet  ->  (x - 0.5)/0.5, per channel affine
    TRANSFORM_SCALE = (0.229 / 0.5, 0.224 / 0.5, 0.225 / 0.5)
    TRANSFORM_SHIFT = ((0.485 - 0.5) / 0.5, (0.456 - 0.5) / 0.5, (0.406 - 0.5) / 0.5)

    def input_spec(self):
        """(space-to-depth stem input, per-channel scale, shift): transform_input folded into the loaders'
        one-pass uint8 conversion (ops/hip.py input_from_u8)."""
        if self.transform_input:
            return (False, self.TRANSFORM_SCALE, self.TRANSFORM_SHIFT)
        return (False, None, None)

    def _transform_input(self, x):
        if not self.transform_input:
            return Fx.prepare_input(x)
        if Fx.use_hip(x):
            return Fx._hip().prepare_input(x, self.TRANSFORM_SCALE, self.TRANSFORM_SHIFT)
        sc = torch.tensor(self.TRANSFORM_SCALE, dtype=x.dtype, device=x.device).view(1, 3, 1, 1)
        sh = torch.tensor(self.TRANSFORM_SHIFT, dtype=x.dtype, device=x.device).view(1, 3, 1, 1)
        return x * sc + sh

    def forward(self, x):
        x = self._transform_input(x)
        x = self.Conv2d_1a_3x3(x)
        x = self.Conv2d_2a_3x3(x, True)
        x = self.Conv2d_2b_3x3(x, True, pool=(3, 2, 0))
        x = self.Conv2d_3b_1x1(x)
        x = self.Conv2d_4a_3x3(x, True, pool=(3, 2, 0))
        x = self.Mixed_5b(x)
        x = self.Mixed_5c(x)
        x = self.Mixed_5d(x)
        x = self.Mixed_6a(x)
        x = self.Mixed_6b(x)
        x = self.Mixed_6c(x)
        x = self.Mixed_6d(x)
        x = self.Mixed_6e(x)
        aux = self.AuxLogits(x) if (self.AuxLogits is not None and self.training) else None
        x = self.Mixed_7a(x)
        x = self.Mixed_7b(x)
        x = self.Mixed_7c(x)
        x = Fx.global_avg_pool(x)
        x = Fx.dropout(x, self.dropout.p, self.training)
        x = Fx.mlp(x, self.fc) if isinstance(self.fc, nn.Sequential) else Fx.linear(x, self.fc)
        if self.training and self.aux_logits:
            return InceptionOutputs(x, aux)
        return x


def inception_v3(num_classes=1000, aux_logits=True, transform_input=False):
    return Inception3(num_classes=num_classes, aux_logits=aux_logits, transform_input=transform_input)
