"""The ResNet stem convolution (space-to-depth form: 4x4 stride-1 over 16 channels, 64 outputs) in
isolation: every implicit-GEMM kernel configuration and the direct halo-tile kernel, with and without the fused BN-statistics epilogue, against its
roofline (output write + input read at 6 TB/s; FLOPs at 2.3 PF).

    python benchmarks/stem_bench.py --batch 512
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()
    from pytorch_imageclassification_distributed_amd.ops import hip
    C = hip.C
    n, h = a.batch, 224
    dev = "cuda"
    x = torch.randn(n, 3, h, h, device=dev)
    xs = hip._empty_cl(n, 16, h // 2, h // 2, dev)
    C.prepare_input_s2d(x, xs, n, h, h)
    g = hip._s2d_geom(n, h, h, 64)
    wq = (torch.randn(64, 256, device=dev) * 0.05).to(torch.bfloat16).view(-1)
    y = hip._empty_cl(n, 64, h // 2, h // 2, dev)
    dh, dw, tb = hip._fwd_taps(g)
    m = g.N * g.OH * g.OW
    geo = (m, g.Co, g.T * g.Cx, g.Cx, g.OH, g.OW, g.H, g.W, 1, g.T * g.Cx, g.OH, g.OW, 1, 0, 0, 64, 0)
    grp = hip.stat_groups(m)
    stats = torch.zeros(grp * 2 * 64, device=dev)
    zero = hip.ws(torch.device(dev)).zero
    roof_us = max(2.0 * m * 64 * 256 / 2.3e15, (m * 64 * 2 + xs.numel() * 2) / 6e12) * 1e6
    print(f"stem M={m} N=64 K=256: roofline {roof_us:.0f} us")
    for i, cfg in enumerate(hip.conv_cfgs()):
        if cfg[1] != 64:
            continue
        for st in (None, stats):
            t = timeit(lambda: C.conv_gemm(xs, wq, y, st, None, *geo, dh, dw, tb, grp, zero, None,
                                           None, None, None, None, 0, 1, 0, 0, i, None, None, None, None, None, None, None, 0, None, None, None, None, 0))
            print(f"  cfg {cfg}: {'stats' if st is not None else 'plain'} {t:7.1f} us  "
                  f"{(m * 64 * 2 + xs.numel() * 2) / t / 1e6:5.2f} TB/s")
    for st in (None, stats):
        t = timeit(lambda: C.stem_conv(xs, wq, y, st, grp, n, h // 2, h // 2))
        print(f"  direct halo-tile kernel (stem.hip): {'stats' if st is not None else 'plain'} {t:7.1f} us  "
              f"{(m * 64 * 2 + xs.numel() * 2) / t / 1e6:5.2f} TB/s")
    y2 = torch.empty_like(y)
    t = timeit(lambda: y2.copy_(y))
    print(f"  copy of the output tensor: {t:7.1f} us ({2 * y.numel() * 2 / t / 1e6:.2f} TB/s)")


if __name__ == "__main__":
    main()
