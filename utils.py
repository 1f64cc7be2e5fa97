"""Reference-compatible facade for ``utils`` (reference utils.py): AverageMeter, Accuracy."""
from pytorch_imageclassification_distributed_amd.utils.meters import Accuracy, AverageMeter

__all__ = ["AverageMeter", "Accuracy"]
