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
* ``HostSyntheticLoader`` - the host data path of a real run (K24/K25) with the
  decode left out: a ring of *pinned* uint8 NHWC batches (what the native
  loader's C++ workers produce, data/native.py) is copied to the GPU with
  ``hipMemcpyAsync`` on a copy stream, one batch ahead, and converted there -
  with ``input_fn`` set (the trainer's, HIP path) straight to the model's bf16
  input in one kernel (``input_from_u8``), else normalised to fp32 NCHW
  (``normalize_u8``); the compute stream waits on an event.  ``bench.py --data
  host`` times the training step with it, so the H2D copy and normalisation the
  on-device loader skips are inside the measurement.
"""
from __future__ import annotations

import torch
from torch.utils.data import Dataset

from .prefetch import copy_stream


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


class HostSyntheticLoader:
    """Pinned uint8 host batches -> copy stream -> on-device normalisation, double-buffered (see module
    docstring).  Iterating yields ``{'image': fp32 NCHW, 'label': int64}`` ready on the current stream."""

    def __init__(self, batch_size: int, num_classes: int, image_size: int, device, steps: int,
                 ring: int = 2, seed: int = 0):
        from .. import _ext
        self.C = _ext.load()
        g = torch.Generator().manual_seed(seed)
        self.host = []
        for _ in range(max(ring, 2)):
            img = torch.randint(0, 256, (batch_size, image_size, image_size, 3), dtype=torch.uint8,
                                generator=g).pin_memory()
            lab = torch.randint(0, num_classes, (batch_size,), generator=g).pin_memory()
            self.host.append((img, lab))
        self.device = torch.device(device)
        self.stream = copy_stream(self.device)
        self.steps = steps
        self.input_fn = None  # as NativeFolderLoader.input_fn: uint8 -> model input in one pass, on the copy stream

    def __len__(self):
        return self.steps

    def _issue(self, i):
        from .folder import IMAGENET_MEAN, IMAGENET_STD
        img, lab = self.host[i % len(self.host)]
        n, s = img.shape[0], img.shape[1]
        with torch.cuda.stream(self.stream):
            u8 = img.to(self.device, non_blocking=True)
            y = lab.to(self.device, non_blocking=True)
            if self.input_fn is not None:
                x = self.input_fn(u8)
            else:
                x = torch.empty((n, 3, s, s), dtype=torch.float32, device=self.device)
                self.C.normalize_u8(u8, x, list(IMAGENET_MEAN), list(IMAGENET_STD))
        return {"image": x, "label": y, "_u8": u8}

    def __iter__(self):
        cur = torch.cuda.current_stream(self.device)
        nxt = self._issue(0) if self.steps > 0 else None
        for i in range(self.steps):
            b = nxt
            cur.wait_stream(self.stream)
            for t in b.values():
                t.record_stream(cur)
            # the next batch's copy + normalisation overlap this step (the pinned source slot it reads is
            # not written again: the ring is read-only host memory)
            nxt = self._issue(i + 1) if i + 1 < self.steps else None
            yield {"image": b["image"], "label": b["label"]}

    def set_epoch(self, epoch: int) -> None:
        pass
