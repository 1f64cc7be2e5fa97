"""Reference-compatible facade for ``dp/loader.py``: ``ImageDataset(data_dir, fold, resize_size)``.

Implementation: ``pytorch_imageclassification_distributed_amd.data.folder``.
"""
from pytorch_imageclassification_distributed_amd.data.folder import (ImageDataset, brightness,
                                                                     contrast, saturation)
from pytorch_imageclassification_distributed_amd.data.synthetic import SyntheticImageDataset

__all__ = ["ImageDataset", "SyntheticImageDataset", "saturation", "brightness", "contrast"]
