from .config import REF_CLASS_WEIGHTS, build_parser, parse_class_weights
from .optim import FusedAdam, MultiStepLR
from .trainer import Trainer

__all__ = ["Trainer", "FusedAdam", "MultiStepLR", "build_parser", "parse_class_weights",
           "REF_CLASS_WEIGHTS"]
