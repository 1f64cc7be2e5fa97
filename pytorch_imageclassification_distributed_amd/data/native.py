"""Native (C++) image-folder loader: the drop-in replacement for the reference's DataLoader.

Reference: ``DataLoader(ImageDataset(...), batch_size=B, sampler=DistributedSampler, num_workers=6,
pin_memory=True)`` (train.py:112-118) running dp/loader.py's per-sample Python preprocessing in
worker processes.

Here ``csrc/loader.cpp`` does the per-sample work in C++ threads (PNG decode with zlib, nearest
resize, the reference augmentation) straight into a ring of pinned uint8 NHWC batch slots.  The
Python side:
* takes this rank's indices from the same ``DistributedSampler`` (so sharding, per-epoch shuffling
  and padding are the reference's),
* copies each slot to the GPU as uint8 on a dedicated copy stream (a quarter of the fp32 bytes),
* normalises on the GPU with one kernel into the fp32 NCHW batch the models consume
  (``normalize_u8``: (x/255 - mean) / std, dp/loader.py:86-91),
* hands a slot back to the C++ workers once the copy that reads it has completed.

Batches are dicts ``{'image': fp32 [n,3,S,S], 'label': int64 [n]}`` on the target device (CPU: the
worker threads write the normalised fp32 batch themselves).  PNG only (the reference reads PNG files, ``image_id`` strips ``.png``);
``use_native()`` tells whether a dataset qualifies.
"""
from __future__ import annotations

from collections import deque

import torch

from .folder import IMAGENET_MEAN, IMAGENET_STD, ImageDataset
from .prefetch import copy_stream


def available() -> bool:
    try:
        from .. import _ext
        return hasattr(_ext.load(), "NativeLoader")
    except Exception:  # noqa: BLE001  (no extension built: the Python loader is used)
        return False


def use_native(ds) -> bool:
    return (isinstance(ds, ImageDataset) and len(ds) > 0
            and all(f.lower().endswith(".png") for f in ds.image_files) and available())


class NativeFolderLoader:
    def __init__(self, dataset: ImageDataset, sampler, batch_size: int, device, workers: int = 6,
                 augment: bool | None = None, drop_last: bool = False, ring: int = 4, seed: int = 0):
        from .. import _ext
        C = _ext.load()
        self.ds, self.sampler, self.batch_size = dataset, sampler, batch_size
        self.device = torch.device(device)
        self.drop_last = drop_last
        aug = (dataset.fold == "train" and dataset.augment_train) if augment is None else augment
        labels = [dataset.mapping[f.replace("\\", "/").split("/")[-2]] for f in dataset.image_files]
        cuda = self.device.type == "cuda"
        self.core = C.NativeLoader(list(dataset.image_files), labels, dataset.resize_size, batch_size,
                                   max(int(workers), 1), bool(aug), int(seed), int(ring), cuda, not cuda,
                                   list(IMAGENET_MEAN), list(IMAGENET_STD))
        self.C = C
        self.stream = copy_stream(self.device) if cuda else None
        self.epoch = 0
        self.ring = max(int(ring), 2)
        self._pending: deque = deque()
        # optional uint8 NHWC (device) -> model input conversion run on the copy stream (the trainer sets it
        # on the HIP path: normalisation + layout + transform_input in one kernel); None = fp32 NCHW batches
        self.input_fn = None

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
        if hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(epoch)

    def __len__(self):
        n = len(self.sampler) if self.sampler is not None else len(self.ds)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def _drain(self, block: bool, keep: int = 0) -> None:
        """Return slots whose host->device copy has finished; when ``block``, wait until at most
        ``keep`` slots are still out (batch c reuses batch c-ring's slot)."""
        while len(self._pending) > keep:
            slot, ev = self._pending[0]
            if ev is not None and not (block or ev.query()):
                break
            if ev is not None:
                ev.synchronize()
            self.core.release(slot)
            self._pending.popleft()

    def _to_device(self, slot, img_u8, labels):
        if self.stream is None:  # CPU: the worker threads already wrote the normalised fp32 batch
            self._pending.append((slot, None))
            return {"image": img_u8.clone(), "label": labels.clone()}
        cur = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self.stream):
            u8 = img_u8.to(self.device, non_blocking=True)
            lab = labels.to(self.device, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
            if self.input_fn is not None:  # the model's first-layer input in one pass (ops/hip.py input_from_u8)
                x = self.input_fn(u8)
            else:
                n, s = img_u8.shape[0], img_u8.shape[1]
                x = torch.empty((n, 3, s, s), dtype=torch.float32, device=self.device)
                self.C.normalize_u8(u8, x, list(IMAGENET_MEAN), list(IMAGENET_STD))
        cur.wait_stream(self.stream)
        for t in (u8, lab, x):
            t.record_stream(cur)
        self._pending.append((slot, ev))
        return {"image": x, "label": lab}

    def __iter__(self):
        self._drain(block=True)
        order = list(iter(self.sampler)) if self.sampler is not None else list(range(len(self.ds)))
        # the augmentation stream follows the sampler's epoch (the trainer calls sampler.set_epoch)
        epoch = getattr(self.sampler, "epoch", self.epoch)
        self.core.start_epoch(order, int(epoch), self.drop_last)
        try:
            while True:
                self._drain(block=False)
                self._drain(block=True, keep=self.ring - 1)
                got = self.core.next()
                if got is None:
                    break
                slot, img, lab = got
                yield self._to_device(slot, img, lab)
        finally:
            self._drain(block=True)


def decode_preprocess(path: str, size: int, augment: bool = False, seed: int = 0, epoch: int = 0,
                      index: int = 0) -> torch.Tensor:
    """One image through the native decode + preprocessing path (uint8 [S,S,3])."""
    from .. import _ext
    return _ext.load().decode_preprocess(path, size, augment, seed, epoch, index)
