"""Image-folder loading throughput: native C++ loader vs the reference-style Python DataLoader.

Writes a synthetic PNG folder (ImageNet-like 256x256 RGB by default, reference layout
<root>/train/<class>/*.png), then times full passes of each loader producing fp32 NCHW batches
(train-fold augmentation on, nearest resize to --size).

    python benchmarks/loader_bench.py --images 2048 --workers 8 [--device cuda]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_folder(root, n, hw, classes=7):
    from PIL import Image
    rng = np.random.default_rng(0)
    for i in range(n):
        d = os.path.join(root, "train", f"c{i % classes}")
        os.makedirs(d, exist_ok=True)
        # smooth-ish content so PNG compression is realistic (pure noise would not compress)
        base = rng.integers(0, 256, (hw // 8, hw // 8, 3), dtype=np.uint8)
        img = np.kron(base, np.ones((8, 8, 1), dtype=np.uint8)) + rng.integers(0, 8, (hw, hw, 3), dtype=np.uint8)
        Image.fromarray(img).save(os.path.join(d, f"img_{i}.png"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=2048)
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--workers", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--device", default="cpu")
    ap.add_argument("--root", default="")
    a = ap.parse_args()
    import torch
    from torch.utils.data import DataLoader
    from pytorch_imageclassification_distributed_amd.data import ImageDataset, NativeFolderLoader
    root = a.root or tempfile.mkdtemp(prefix="imgcls_loader_")
    if not os.path.isdir(os.path.join(root, "train")):
        make_folder(root, a.images, a.hw)
    ds = ImageDataset(root, "train", a.size)
    res = {"images": len(ds), "hw": a.hw, "size": a.size, "workers": a.workers, "device": a.device}

    def run(loader, to_dev):
        t0 = time.perf_counter()
        n = 0
        for b in loader:
            x = b["image"]
            if to_dev and x.device.type != a.device:
                x = x.to(a.device, non_blocking=True)
            n += x.shape[0]
        if a.device == "cuda":
            torch.cuda.synchronize()
        return n / (time.perf_counter() - t0)

    # decode + resize + augment into the pinned uint8 ring only (the C++ worker threads)
    labels = [ds.mapping[f.replace("\\", "/").split("/")[-2]] for f in ds.image_files]
    from pytorch_imageclassification_distributed_amd import _ext
    core = _ext.load().NativeLoader(ds.image_files, labels, a.size, a.batch, a.workers, True, 0, 4, False, False)
    for rep in range(2):
        core.start_epoch(list(range(len(ds))), rep, False)
        t0, n = time.perf_counter(), 0
        while (got := core.next()) is not None:
            n += got[1].shape[0]
            core.release(got[0])
        res["native_core_img_per_s"] = round(n / (time.perf_counter() - t0), 1)
    nat = NativeFolderLoader(ds, None, a.batch, a.device, workers=a.workers)
    run(nat, False)  # warm file cache
    res["native_img_per_s"] = round(run(nat, False), 1)
    py = DataLoader(ds, batch_size=a.batch, num_workers=a.workers, pin_memory=a.device == "cuda")
    res["python_img_per_s"] = round(run(py, True), 1)
    res["speedup"] = round(res["native_img_per_s"] / res["python_img_per_s"], 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
