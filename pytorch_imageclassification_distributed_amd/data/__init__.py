from .folder import (IMAGENET_MEAN, IMAGENET_STD, ImageDataset, augment, brightness, contrast,
                     normalize, resize_nearest, saturation)
from .native import NativeFolderLoader, use_native
from .prefetch import CudaPrefetcher
from .synthetic import DeviceSyntheticLoader, HostSyntheticLoader, SyntheticImageDataset

__all__ = [
    "ImageDataset", "SyntheticImageDataset", "NativeFolderLoader", "use_native", "DeviceSyntheticLoader", "HostSyntheticLoader", "CudaPrefetcher",
    "augment", "normalize", "resize_nearest", "saturation", "brightness", "contrast",
    "IMAGENET_MEAN", "IMAGENET_STD",
]
