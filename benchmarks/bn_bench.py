"""BatchNorm elementwise kernels (apply fwd, backward elementwise) on the ResNet-50 BN shapes: achieved
HBM bandwidth (apply moves 3 bf16 tensors incl. the residual, backward 4).

The row reductions (bwd reduce, stats) are swept over block count x channel-chunk lanes per block.

A channel-group-stationary variant (each thread pinned to one 8-channel group, coefficients in
registers, two rows in flight) was measured slower than these flat grid-stride kernels (11.3 vs 10.1 ms
of backward per ResNet-50 step at batch 512) and removed.

    python benchmarks/bn_bench.py --batch 512
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (C, H) of ResNet-50 BN outputs (with how many layers share the shape)
SHAPES = [(32, 112, 1), (96, 112, 1), (64, 112, 1), (64, 56, 6), (256, 56, 4), (128, 56, 1), (128, 28, 7), (512, 28, 5), (256, 28, 1),
          (256, 14, 11), (1024, 14, 7), (512, 14, 1), (512, 7, 5), (2048, 7, 4)]


def timeit(fn, iters=20):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()
    from pytorch_imageclassification_distributed_amd.ops import hip
    C = hip.C
    dev = "cuda"
    out = []
    tot = [0.0, 0.0]
    for (c, h, cnt) in SHAPES:
        rows = a.batch * h * h
        y = torch.randn(rows * c, device=dev).to(torch.bfloat16)
        g = torch.randn(rows * c, device=dev).to(torch.bfloat16)
        res = torch.randn(rows * c, device=dev).to(torch.bfloat16)
        o = torch.empty_like(y)
        coef = torch.rand(4 * c, device=dev) + 0.5
        kk = torch.randn(2 * c, device=dev) * 0.01
        row = {"C": c, "H": h}
        ta = timeit(lambda: C.bn_apply(y, coef, res, o, rows, c, c, 0, 1, None, None))
        tb = timeit(lambda: C.bn_bwd_elemt(g, y, coef, kk, res, None, o, rows, c, 1))
        nbytes = rows * c * 2
        row["apply_us"] = round(ta * 1e3, 1)
        row["apply_TBps"] = round(3 * nbytes / ta / 1e9, 2)
        row["bwd_us"] = round(tb * 1e3, 1)
        row["bwd_TBps"] = round(4 * nbytes / tb / 1e9, 2)
        tot[0] += ta * cnt
        tot[1] += tb * cnt
        part = torch.zeros(64 * 2 * c, device=dev)
        for nb in (1024, 2048):
            for chb in (8, 32, 256):  # channel-chunk lanes per block (32 = default; 256 = the former layout)
                if chb > 8 and chb > c // 8:
                    continue
                C.bn_set_reduce_blocks(nb, chb)
                tr = timeit(lambda: C.bn_bwd_reduce(g, y, coef, res, o, rows, c, 1, part, 64))
                ts = timeit(lambda: C.bn_stats(y, rows, c, part, 64))
                row[f"bwdred{nb}_chb{chb}_us"] = round(tr * 1e3, 1)
                row[f"stats{nb}_chb{chb}_us"] = round(ts * 1e3, 1)
        C.bn_set_reduce_blocks(0, 0)
        print(row, flush=True)
        out.append(row)
    print(json.dumps({"batch": a.batch, "total_ms_apply_bwd": [round(x, 3) for x in tot]}))


if __name__ == "__main__":
    main()
