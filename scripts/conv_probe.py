"""Run ONE convolution GEMM of a ResNet-50 layer repeatedly (for rocprofv3 --pmc / --kernel-trace passes).

    python scripts/conv_probe.py --shape 128,128,3,1,1,28 --batch 1024 --op fwd --cfg 1 --iters 20

``--cfg``: index into ``ops.hip.conv_cfgs()`` (fwd / dgrad), forced for every launch (-1: tuned choice);
``--halo``: index into ``ops.hip.conv_halo_cfgs()`` instead (the halo-patch kernel; stride-1 3x3 window);
``--op``: fwd | dgrad | wgrad (wgrad: ``--wstages`` forces the ring / tile variant).  Prints the mean
time per launch and the TF/s of the GEMM.  Synthetic bf16 data, random weights.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="128,128,3,1,1,28", help="Cin,Cout,k,stride,pad,H_in")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--op", default="fwd", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--cfg", type=int, default=-1)
    ap.add_argument("--halo", type=int, default=-1)
    ap.add_argument("--deep", type=int, default=-1, help="index into ops.hip.conv_deep_cfgs() (prefetch-depth-2 kernel)")
    ap.add_argument("--direct", type=int, default=-1, help="index into ops.hip.DIRECT_CFGS (halo-tile direct kernels)")
    ap.add_argument("--pw", type=int, default=-1, help="index into ops.hip.conv_pw_cfgs() (1x1 resident-weight kernel)")
    ap.add_argument("--wstages", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from pytorch_imageclassification_distributed_amd.ops import hip
    cin, cout, k, s, p, h = (int(v) for v in a.shape.split(","))
    dev = torch.device("cuda")
    torch.manual_seed(0)
    conv = nn.Conv2d(cin, cout, k, s, p, bias=False).to(dev).to(memory_format=torch.channels_last)
    x = torch.randn(a.batch, cin, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    if a.cfg >= 0:
        hip.CONV_FORCE_CFG = (0, 0, a.cfg)
    if a.halo >= 0:
        hip.HALO_FORCE = a.halo
    if a.deep >= 0:
        hip.DEEP_FORCE = a.deep
    if a.direct >= 0:
        hip.DIRECT_FORCE = a.direct
    if a.pw >= 0:
        hip.PW_FORCE = a.pw
    if a.wstages:
        hip.WGRAD_STAGES = a.wstages
    hip.ensure_channels_last_weight(conv)
    g = hip.conv_geom(x, conv)
    y = hip.conv_forward_raw(x, conv.weight, g)
    dy = torch.randn_like(y)
    if a.op == "fwd":
        run = lambda: hip.conv_forward_raw(x, conv.weight, g)  # noqa: E731
    elif a.op == "dgrad":
        run = lambda: hip.conv_dgrad_raw(dy, conv.weight, g)  # noqa: E731
    else:
        dw = torch.zeros(cout * g.T * g.Cx, dtype=torch.float32, device=dev)
        m, ntot = g.N * g.OH * g.OW, g.T * g.Cx
        kps, splits, st = hip._wgrad_plan(g, dy, x, m, ntot)
        run = lambda: hip._wgrad_launch(dy, x, dw, g, m, ntot, kps, splits, st)  # noqa: E731
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    flops = 2.0 * g.N * g.OH * g.OW * cout * g.T * cin
    tag = f"halo {a.halo}" if a.halo >= 0 else f"direct {a.direct}" if a.direct >= 0 else \
        f"pw {a.pw}" if a.pw >= 0 else f"cfg {a.cfg}"
    print(f"{a.op} shape {a.shape} b{a.batch} {tag}: {ms * 1e3:.1f} us  {flops / ms / 1e9:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
