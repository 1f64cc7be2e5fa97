from .folder import (IMAGENET_MEAN, IMAGENET_STD, ImageDataset, augment, brightness, contrast,
                     normalize, resize_nearest, saturation)
from .prefetch import CudaPrefetcher
from .synthetic import DeviceSyntheticLoader, SyntheticImageDataset

__all__ = [
    "ImageDataset", "SyntheticImageDataset", "DeviceSyntheticLoader", "CudaPrefetcher",
    "augment", "normalize", "resize_nearest", "saturation", "brightness", "contrast",
    "IMAGENET_MEAN", "IMAGENET_STD",
]
