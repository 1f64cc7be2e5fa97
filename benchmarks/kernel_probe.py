"""Run ONE convolution kernel of one ResNet-50 shape repeatedly (for rocprofv3 --pmc passes and
per-kernel timing): forward / data-gradient with a fixed configuration, or weight-gradient with a fixed
(split target, variant).

    python benchmarks/kernel_probe.py --shape 0 --mode fwd --cfg 5 [--batch 512] [--iters 5]
    python benchmarks/kernel_probe.py --shape 0 --mode wgrad --wblocks 512 --wstages 1
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.conv_bench import R50  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, default=0)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--mode", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--cfg", type=int, default=-1, help="conv configuration index (fwd / dgrad)")
    ap.add_argument("--wblocks", type=int, default=512)
    ap.add_argument("--wstages", type=int, default=1)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from pytorch_imageclassification_distributed_amd.ops import hip
    dev = "cuda"
    ci, co, k, s, p, h, _cnt = R50[a.shape]
    torch.manual_seed(0)
    conv = nn.Conv2d(ci, co, k, s, p, bias=False).to(dev).to(memory_format=torch.channels_last)
    x = torch.randn(a.batch, ci, h, h, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = hip.ConvGeom(x, conv)
    hip.CONV_FORCE_CFG = (0, 0, a.cfg) if a.cfg >= 0 else None
    hip.WGRAD_TARGET_BLOCKS, hip.WGRAD_STAGES = a.wblocks, a.wstages
    stats = hip.ws(x.device).stats_buf(co)
    y = hip.conv_forward_raw(x, conv.weight, g, stats=stats)
    dy = torch.randn_like(y)
    if a.mode == "fwd":
        run = lambda: hip.conv_forward_raw(x, conv.weight, g, stats=stats)  # noqa: E731
    elif a.mode == "dgrad":
        run = lambda: hip.conv_dgrad_raw(dy, conv.weight, g)  # noqa: E731
    else:
        run = lambda: hip.conv_wgrad_raw(dy, x, conv.weight, g)  # noqa: E731
    run()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(a.iters):
        run()
    ev[1].record()
    ev[1].synchronize()
    ms = ev[0].elapsed_time(ev[1]) / a.iters
    macs = a.batch * g.OH * g.OW * co * ci * k * k
    print(f"shape {a.shape} ({ci}->{co} k{k}s{s} {h}x{h}) {a.mode} cfg {a.cfg}: {ms * 1e3:.1f} us "
          f"{2 * macs / ms / 1e9:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
