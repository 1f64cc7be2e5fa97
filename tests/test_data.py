"""Dataset / augmentation / sampler behaviour (reference dp/loader.py, train.py:112-118)."""
import random

import numpy as np
import pytest
import torch
from PIL import Image, ImageEnhance
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler

from pytorch_imageclassification_distributed_amd.data import (IMAGENET_MEAN, IMAGENET_STD, ImageDataset,
                                                              SyntheticImageDataset, augment, brightness,
                                                              contrast, normalize, resize_nearest, saturation)


@pytest.fixture()
def folder(tmp_path):
    rng = np.random.RandomState(0)
    for fold, n in (("train", 3), ("valid", 2)):
        for cls in ("cat", "dog", "emu"):
            d = tmp_path / fold / cls
            d.mkdir(parents=True)
            for i in range(n):
                arr = rng.randint(0, 255, (20 + i, 17, 4), dtype=np.uint8)
                Image.fromarray(arr, "RGBA").save(d / f"{cls}_{i}.png")
    return tmp_path


def test_imagefolder_mapping_and_sample(folder):
    ds = ImageDataset(str(folder), "train", 16)
    assert ds.num_classes == 3 and ds.mapping == {"cat": 0, "dog": 1, "emu": 2}
    assert len(ds) == 9
    assert ds.image_files == sorted(ds.image_files)  # deterministic order (defect A4)
    s = ds[4]
    assert set(s) == {"image", "label", "image_id"}
    assert s["image"].shape == (3, 16, 16) and s["image"].dtype == torch.float32
    assert s["image_id"] == "dog_1" and s["label"] == 1


def test_valid_fold_is_not_augmented(folder):
    ds = ImageDataset(str(folder), "valid", 12)
    a, b = ds[0]["image"], ds[0]["image"]
    assert torch.equal(a, b)
    raw = np.asarray(Image.open(ds.image_files[0]))[..., :3]
    ref = normalize(resize_nearest(raw, 12)).transpose(2, 0, 1)
    assert np.allclose(a.numpy(), ref, atol=1e-6)


def test_normalize_matches_reference_formula():
    img = np.random.RandomState(1).randint(0, 255, (4, 5, 3), dtype=np.uint8)
    out = normalize(img)
    exp = img.astype(np.float32) / 255
    for i in range(3):
        exp[..., i] = (exp[..., i] - IMAGENET_MEAN[i]) / IMAGENET_STD[i]
    assert np.allclose(out, exp, atol=1e-6)


def test_resize_nearest_index_rule():
    img = np.arange(6 * 4).reshape(6, 4, 1).astype(np.uint8)
    out = resize_nearest(img, 3)
    assert out[:, :, 0].tolist() == [[0, 1, 2], [8, 9, 10], [16, 17, 18]]


@pytest.mark.parametrize("fn,enh", [(saturation, ImageEnhance.Color), (brightness, ImageEnhance.Brightness),
                                    (contrast, ImageEnhance.Contrast)])
def test_jitter_matches_pil(fn, enh):
    img = np.random.RandomState(2).randint(0, 255, (16, 16, 3), dtype=np.uint8)
    for f in (0.9, 1.07):
        ours = fn(img, f).astype(int)
        ref = np.asarray(enh(Image.fromarray(img)).enhance(f)).astype(int)
        assert np.abs(ours - ref).max() <= 2


def test_augment_geometry_and_determinism():
    img = np.random.RandomState(3).randint(0, 255, (8, 8, 3), dtype=np.uint8)
    a = augment(img, random.Random(5))
    b = augment(img, random.Random(5))
    assert a.shape == (8, 8, 3) and np.array_equal(a, b)


def test_distributed_sampler_shards_disjoint_and_padded():
    ds = SyntheticImageDataset(10, 3, 8)
    shards = [list(DistributedSampler(ds, num_replicas=3, rank=r, seed=0)) for r in range(3)]
    assert all(len(s) == 4 for s in shards)  # ceil(10/3), padded
    flat = sum(shards, [])
    assert set(flat) == set(range(10)) and len(flat) == 12


def test_synthetic_dataset_loader():
    ds = SyntheticImageDataset(12, 4, 8)
    batch = next(iter(DataLoader(ds, batch_size=4)))
    assert batch["image"].shape == (4, 3, 8, 8) and batch["label"].tolist() == [0, 1, 2, 3]
    assert torch.equal(ds[3]["image"], ds[3]["image"])
