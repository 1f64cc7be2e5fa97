from .classifier import DEFAULT_IMAGE_SIZE, MODEL_NAMES, Classifier, build_backbone, mlp_head
from .efficientnet import EfficientNet, efficientnet, efficientnet_b0, efficientnet_b3
from .inception import Inception3, InceptionOutputs, inception_v3
from .resnet import ResNet, resnet18, resnet34, resnet50, resnet101, resnet152

__all__ = [
    "Classifier", "build_backbone", "mlp_head", "MODEL_NAMES", "DEFAULT_IMAGE_SIZE",
    "ResNet", "resnet18", "resnet34", "resnet50", "resnet101", "resnet152",
    "Inception3", "InceptionOutputs", "inception_v3",
    "EfficientNet", "efficientnet", "efficientnet_b0", "efficientnet_b3",
]
