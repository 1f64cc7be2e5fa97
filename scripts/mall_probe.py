"""Does image-chunking a conv's backward keep its operands in the 256 MB Infinity Cache?

A conv's data gradient and weight gradient both read dY (and the weight gradient reads X).  Run back to
back over the whole batch, the second read of a 1.6 GB dY comes from HBM.  Run per chunk of images
(dgrad(chunk) then wgrad(chunk)), the chunk's dY may still be on-die when the weight gradient reads it.
This times both orders on one stream for one ResNet-50 layer shape:

    python scripts/mall_probe.py --shape 64,256,1,1,0,56 --batch 1024 --chunks 1,4,8,16,32
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
    ap.add_argument("--shape", default="64,256,1,1,0,56", help="Cin,Cout,k,stride,pad,H_in")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--chunks", default="1,4,8,16,32")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from pytorch_imageclassification_distributed_amd.ops import hip
    cin, cout, k, s, p, h = (int(v) for v in a.shape.split(","))
    dev = torch.device("cuda")
    torch.manual_seed(0)
    conv = nn.Conv2d(cin, cout, k, s, p, bias=False).to(dev).to(memory_format=torch.channels_last)
    hip.ensure_channels_last_weight(conv)
    x = torch.randn(a.batch, cin, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = hip.conv_geom(x, conv)
    y = hip.conv_forward_raw(x, conv.weight, g)
    dy = torch.randn_like(y)
    dw = torch.zeros(cout * g.T * g.Cx, dtype=torch.float32, device=dev)
    nbytes = (dy.numel() + x.numel()) * 2

    def run(nch):
        step = a.batch // nch
        for i0 in range(0, a.batch, step):
            xc, dyc = x[i0:i0 + step], dy[i0:i0 + step]
            gc = hip.conv_geom(xc, conv)
            hip.conv_dgrad_raw(dyc, conv.weight, gc)
            m, ntot = gc.N * gc.OH * gc.OW, gc.T * gc.Cx
            kps, splits, st = hip._wgrad_plan(gc, dyc, xc, m, ntot)
            hip._wgrad_launch(dyc, xc, dw, gc, m, ntot, kps, splits, st)

    for nch in (int(v) for v in a.chunks.split(",")):
        if a.batch % nch:
            continue
        for _ in range(3):
            run(nch)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            run(nch)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        print(f"mall {a.shape} b{a.batch} chunks {nch:3d} ({a.batch // nch} img, dY {dy.numel() * 2 / nch / 2**20:.0f} MiB): "
              f"dgrad+wgrad {ms * 1e3:.1f} us  ({nbytes / ms / 1e9:.2f} TB/s of dY+X)", flush=True)


if __name__ == "__main__":
    main()
