"""ResNet-18/34/50/101/152 (torchvision v1.5 topology and parameter names).

The reference builds these with ``torchvision.models.resnet{50,101}(pretrained=True)``
(reference nn/classifier.py:11-15); torchvision is not available here and
pretrained weights are not fetchable, so the architecture is re-declared with
identical module names (``conv1, bn1, layer{1..4}.{i}.{conv,bn}{1..3},
downsample.{0,1}, fc``) so checkpoints stay key-compatible.

The forward is written against ``ops.functional`` so the GPU path runs the fused
HIP conv->BN->(+identity)->ReLU kernels while the CPU path uses ATen.
"""
from __future__ import annotations

import torch.nn as nn

from ..ops import functional as Fx


def _conv3x3(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 3, stride, 1, bias=False)


def _conv1x1(cin, cout, stride=1):
    return nn.Conv2d(cin, cout, 1, stride, 0, bias=False)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = _conv3x3(inplanes, planes, stride)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = _conv3x3(planes, planes)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        slot = Fx.grad_slot(x)  # x feeds conv1 and the identity/downsample branch
        if self.downsample is not None:
            identity = Fx.conv_bn_act(x, self.downsample[0], self.downsample[1], None, x_slot=slot, defer_res=True)
        else:
            identity = x
        out = Fx.conv_bn_act(x, self.conv1, self.bn1, "relu", x_slot=slot, defer_act=True)
        return Fx.conv_bn_act(out, self.conv2, self.bn2, "relu", residual=identity,
                              res_slot=None if self.downsample is not None else slot, exclusive_input=True)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        width = planes
        self.conv1 = _conv1x1(inplanes, width)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = _conv3x3(width, width, stride)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = _conv1x1(width, planes * self.expansion)
        self.bn3 = nn.BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        slot = Fx.grad_slot(x)  # x feeds conv1 and the identity/downsample branch
        if self.downsample is not None:
            identity = Fx.conv_bn_act(x, self.downsample[0], self.downsample[1], None, x_slot=slot, defer_res=True)
        else:
            identity = x
        # bn1 / bn2 outputs feed only the next conv: the HIP path fuses their apply into that conv's loads
        out = Fx.conv_bn_act(x, self.conv1, self.bn1, "relu", x_slot=slot, defer_act=True)
        out = Fx.conv_bn_act(out, self.conv2, self.bn2, "relu", exclusive_input=True, defer_act=True)
        return Fx.conv_bn_act(out, self.conv3, self.bn3, "relu", residual=identity,
                              res_slot=None if self.downsample is not None else slot, exclusive_input=True)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512 * block.expansion, num_classes)
        for m in self.modules():  # torchvision init
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, block, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                _conv1x1(self.inplanes, planes * block.expansion, stride),
                nn.BatchNorm2d(planes * block.expansion),
            )
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward_features(self, x):
        x = Fx.conv_bn_act(x, self.conv1, self.bn1, "relu", pool=(3, 2, 1))  # conv1-bn1-relu-maxpool
        x = self.layer1(x)
        x = self.layer2(x)
        x = self.layer3(x)
        x = self.layer4(x)
        return Fx.global_avg_pool(x)

    def input_spec(self):
        """(space-to-depth stem input, per-channel scale, shift) of the model's first layer (the loaders'
        one-pass uint8 conversion, ops/hip.py input_from_u8)."""
        return (Fx._hip().stem_s2d_conv(self.conv1), None, None)

    def forward(self, x):
        x = Fx.prepare_input(x, stem=self.conv1)
        x = self.forward_features(x)
        return Fx.mlp(x, self.fc) if isinstance(self.fc, nn.Sequential) else Fx.linear(x, self.fc)


def resnet18(num_classes=1000):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes)


def resnet34(num_classes=1000):
    return ResNet(BasicBlock, [3, 4, 6, 3], num_classes)


def resnet50(num_classes=1000):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes)


def resnet101(num_classes=1000):
    return ResNet(Bottleneck, [3, 4, 23, 3], num_classes)


def resnet152(num_classes=1000):
    return ResNet(Bottleneck, [3, 8, 36, 3], num_classes)
