"""Synthetic data (no datasets are fetchable here; BASELINE configs are synthetic).

* ``SyntheticImageDataset`` - map-style CPU dataset with the reference sample
  dict ``{'image','label','image_id'}``; deterministic per index.  Feeds the
  regular DataLoader + DistributedSampler path (BASELINE config 1,
  ResNet-18 on 32x32 CIFAR-shaped data).
* ``DeviceSyntheticLoader`` - ImageNet-shaped batches generated *on the GPU*
  once (a small ring of distinct batches resident in HBM) and replayed, so the
  benchmark measures the training step, not a host decode pipeline.  Batches
  are fp32 NCHW normalised images like the reference loader emits
  (dp/loader.py:58-59); the model's input-conversion kernel turns them into
  bf16 NHWC inside the timed step.
"""
from __future__ import annotations

import torch
from torch.utils.data import Dataset


class SyntheticImageDataset(Dataset):
    def __init__(self, length: int, num_classes: int, image_size: int, seed: int = 0):
        self.length, self.num_classes, self.image_size, self.seed = length, num_classes, image_size, seed

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + idx)
        label = idx % self.num_classes
        img = torch.randn(3, self.image_size, self.image_size, generator=g)
        img += (label / max(self.num_classes - 1, 1) - 0.5)  # learnable class signal
        return {"image": img, "label": label, "image_id": f"syn_{idx}"}


class DeviceSyntheticLoader:
    def __init__(self, batch_size: int, num_classes: int, image_size: int, device,
                 steps: int, ring: int = 2, seed: int = 0, dtype=torch.float32):
        g = torch.Generator(device=device).manual_seed(seed)
        self.batches = []
        for _ in range(ring):
            img = torch.randn(batch_size, 3, image_size, image_size, device=device, generator=g, dtype=dtype)
            lab = torch.randint(0, num_classes, (batch_size,), device=device, generator=g)
            self.batches.append({"image": img, "label": lab})
        self.steps = steps

    def __len__(self):
        return self.steps

    def __iter__(self):
        for i in range(self.steps):
            yield self.batches[i % len(self.batches)]

    def set_epoch(self, epoch: int) -> None:
        pass
