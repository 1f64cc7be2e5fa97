"""Reference-compatible facade for ``nn/classifier.py``: ``Classifier(name, num_classes)``.

Implementation: ``pytorch_imageclassification_distributed_amd.models.classifier``.
"""
from pytorch_imageclassification_distributed_amd.models.classifier import Classifier

__all__ = ["Classifier"]
