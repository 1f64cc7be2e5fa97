"""ImageFolder-style dataset with the reference's preprocessing and augmentation.

Reference: ``ImageDataset(data_dir, fold, resize_size)`` (dp/loader.py:15-91):
* layout ``<data_dir>/<fold>/<class>/<file>`` (fold ``train`` / ``valid``);
* decode, drop alpha (``[..., :3]``), nearest-neighbour resize to S x S;
* train-fold augmentation: rot90 by k~U{0..3}, vertical flip p=.5, horizontal
  flip p=.5, then a cascaded photometric jitter with factor U[0.9, 1.1]:
  saturation with p=.05, else brightness p=.05, else contrast p=.05
  (dp/loader.py:63-83);
* ``x/255`` then ImageNet mean/std normalisation (dp/loader.py:86-91);
* returns ``{'image': CHW float32, 'label': int, 'image_id': str}``.

Defects fixed: the class mapping is built from the sorted class
directory names (A3: the reference leaves it empty), the file list is sorted
(A4: the reference shuffles it unseeded per rank, which breaks
DistributedSampler's disjoint sharding), the missing ``bs.dp.augumentation_utils``
jitter ops (A1) and the un-imported cv2 resize (A2) are implemented here with
PIL-ImageEnhance semantics and cv2 INTER_NEAREST index rules.
"""
from __future__ import annotations

import random
from pathlib import Path

import numpy as np
import torch
from torch.utils.data import Dataset

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
IMAGE_EXTS = {".png", ".jpg", ".jpeg", ".bmp", ".tif", ".tiff", ".webp"}


def _blend(img: np.ndarray, other, factor: float) -> np.ndarray:
    out = other + factor * (img.astype(np.float32) - other)
    return np.clip(out, 0, 255).astype(np.uint8)


def _gray(img: np.ndarray) -> np.ndarray:
    # ITU-R 601-2 luma (PIL "L" conversion)
    return img[..., 0] * 0.299 + img[..., 1] * 0.587 + img[..., 2] * 0.114


def saturation(img: np.ndarray, factor: float) -> np.ndarray:
    """Blend with the grayscale image (PIL ImageEnhance.Color)."""
    return _blend(img, _gray(img.astype(np.float32))[..., None], factor)


def brightness(img: np.ndarray, factor: float) -> np.ndarray:
    """Blend with black (PIL ImageEnhance.Brightness)."""
    return _blend(img, np.float32(0.0), factor)


def contrast(img: np.ndarray, factor: float) -> np.ndarray:
    """Blend with the mean gray level (PIL ImageEnhance.Contrast)."""
    mean = np.float32(int(_gray(img.astype(np.float32)).mean() + 0.5))
    return _blend(img, mean, factor)


def resize_nearest(img: np.ndarray, size: int) -> np.ndarray:
    """cv2.resize(..., (size, size), interpolation=INTER_NEAREST) index rule."""
    h, w = img.shape[:2]
    ys = np.minimum((np.arange(size) * (h / size)).astype(np.int64), h - 1)
    xs = np.minimum((np.arange(size) * (w / size)).astype(np.int64), w - 1)
    return img[ys][:, xs]


def augment(image: np.ndarray, rng: random.Random = random) -> np.ndarray:
    k = rng.randrange(4)
    image = np.rot90(image, k=k)
    if rng.random() > 0.5:
        image = image[::-1, ...]
    if rng.random() > 0.5:
        image = image[:, ::-1, ...]
    if rng.random() > 0.95:
        image = saturation(image, 0.9 + rng.random() * 0.2)
    elif rng.random() > 0.95:
        image = brightness(image, 0.9 + rng.random() * 0.2)
    elif rng.random() > 0.95:
        image = contrast(image, 0.9 + rng.random() * 0.2)
    return image


def normalize(image: np.ndarray, mean=IMAGENET_MEAN, std=IMAGENET_STD) -> np.ndarray:
    image = np.asarray(image, dtype=np.float32) / 255.0
    return (image - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)


def read_image(path: str) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        arr = np.asarray(im.convert("RGBA") if im.mode in ("P", "LA", "PA") else im)
    if arr.ndim == 2:
        arr = np.stack([arr] * 3, -1)
    return arr


class ImageDataset(Dataset):
    def __init__(self, data_dir: str, fold: str, resize_size: int, augment_train: bool = True):
        super().__init__()
        self.data_dir = data_dir
        self.image_dir = Path(data_dir) / fold
        classes = sorted(p.name for p in self.image_dir.iterdir() if p.is_dir()) if self.image_dir.is_dir() else []
        self.mapping = {c: i for i, c in enumerate(classes)}
        self.image_files = sorted(str(p) for p in self.image_dir.glob("*/*")
                                  if p.suffix.lower() in IMAGE_EXTS)
        self.fold = fold
        self.resize_size = resize_size
        self.augment_train = augment_train

    def __len__(self):
        return len(self.image_files)

    @property
    def num_classes(self):
        return len(self.mapping.keys())

    def __getitem__(self, idx):
        image_path = self.image_files[idx]
        image_id = Path(image_path).stem
        image = read_image(image_path)
        image = resize_nearest(image[..., :3], self.resize_size)
        label = self.mapping[Path(image_path).parent.name]
        if self.fold == "train" and self.augment_train:
            image = augment(image)
        image = normalize(image)
        image = torch.from_numpy(np.ascontiguousarray(image.transpose((2, 0, 1))))
        return {"image": image, "label": label, "image_id": image_id}

    # reference method names
    def augument(self, image):  # noqa: D401  (sic, dp/loader.py:63)
        return augment(image)

    def normalize(self, image, mean=IMAGENET_MEAN, std=IMAGENET_STD):
        return normalize(image, mean, std)
