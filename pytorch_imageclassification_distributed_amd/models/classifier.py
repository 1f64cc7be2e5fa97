"""``Classifier(name, num_classes)``: backbone + the reference's 4-layer MLP head.

Reference: nn/classifier.py:7-37.  Behavior kept:
* ``self.encoder`` holds the backbone, so checkpoint keys are
  ``[module.]encoder.<torchvision names>`` (reference train.py:179,187).
* the backbone's final ``fc`` is replaced by
  ``Linear(F,128)-ReLU-Linear(128,64)-ReLU-Linear(64,32)-ReLU-Linear(32,C)``
  (nn/classifier.py:26-34); Inception's ``AuxLogits.fc`` becomes
  ``Linear(768, C)`` (nn/classifier.py:22-23).
* ``forward(images) = encoder(images)`` (Inception returns ``(logits, aux)`` in
  train mode).

Fixed defects: EfficientNet's head is ``_fc`` (A5); weights are
random-init by default, ``pretrained`` may name a local torchvision-layout
state_dict (A6).  Extra names beyond the reference's four (``resnet18/34/152``,
``efficientnet-b0..b7``) are accepted.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .efficientnet import EFFICIENTNET_PARAMS, efficientnet
from .inception import inception_v3
from .resnet import resnet18, resnet34, resnet50, resnet101, resnet152

_RESNETS = {"resnet18": resnet18, "resnet34": resnet34, "resnet50": resnet50,
            "resnet101": resnet101, "resnet152": resnet152}

MODEL_NAMES = sorted(list(_RESNETS) + ["inceptionv3"] + list(EFFICIENTNET_PARAMS))

# default training resolution per family (reference hard-codes 299 for inceptionv3, train.py:110)
DEFAULT_IMAGE_SIZE = {**{k: 224 for k in _RESNETS}, "inceptionv3": 299,
                      **{k: v[2] for k, v in EFFICIENTNET_PARAMS.items()}}


def build_backbone(name: str, num_classes: int = 1000) -> nn.Module:
    if name in _RESNETS:
        return _RESNETS[name](num_classes)
    if name in ("inceptionv3", "inception_v3"):
        return inception_v3(num_classes)
    if name in EFFICIENTNET_PARAMS:
        return efficientnet(name, num_classes)
    raise ValueError(f"unknown model {name!r}; choose from {MODEL_NAMES}")


def mlp_head(in_features: int, num_classes: int) -> nn.Sequential:
    return nn.Sequential(
        nn.Linear(in_features, 128, bias=True), nn.ReLU(inplace=True),
        nn.Linear(128, 64, bias=True), nn.ReLU(inplace=True),
        nn.Linear(64, 32, bias=True), nn.ReLU(inplace=True),
        nn.Linear(32, num_classes, bias=True),
    )


class Classifier(nn.Module):
    def __init__(self, name: str, num_classes: int, pretrained: str | None = None):
        super().__init__()
        if num_classes <= 0:
            raise ValueError("num_classes must be positive (reference defect A3 yields 0)")
        self.name = name
        self.encoder = build_backbone(name, 1000)
        if pretrained:
            sd = torch.load(pretrained, map_location="cpu", weights_only=True)
            sd = sd.get("state_dict", sd)
            self.encoder.load_state_dict({k.replace("module.", "").replace("encoder.", ""): v
                                          for k, v in sd.items()}, strict=False)
        if name in ("inceptionv3", "inception_v3"):
            self.encoder.AuxLogits.fc = nn.Linear(self.encoder.AuxLogits.fc.in_features, num_classes)
        head_attr = "_fc" if name in EFFICIENTNET_PARAMS else "fc"
        fc = getattr(self.encoder, head_attr)
        setattr(self.encoder, head_attr, mlp_head(fc.in_features, num_classes))

    def forward(self, images):
        return self.encoder(images)
