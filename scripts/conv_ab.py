"""A/B of fwd / dgrad conv kernels on ResNet-50 shapes, in ONE process (interleaved rounds, guide rule 24).

For every shape and op: the tuner's choice without the prefetch-depth-2 kernels (IMGCLS_DEEP=0 behaviour),
and each deep configuration forced; rounds alternate between the arms and the median is reported.

    python scripts/conv_ab.py [--batch 1024] [--rounds 5] [--shapes 256,256,3,1,1,14 ...]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = ["256,256,3,1,1,14", "512,512,3,1,1,7", "128,128,3,1,1,28", "64,64,3,1,1,56", "256,256,3,2,1,28",
          "1024,256,1,1,0,14", "256,1024,1,1,0,14", "512,2048,1,1,0,7", "2048,512,1,1,0,7", "128,512,1,1,0,28",
          "512,128,1,1,0,28", "64,256,1,1,0,56", "256,64,1,1,0,56"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--ops", default="fwd,dgrad")
    ap.add_argument("--shapes", nargs="*", default=SHAPES)
    a = ap.parse_args()
    from pytorch_imageclassification_distributed_amd.ops import hip
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for shape in a.shapes:
        cin, cout, k, s, p, h = (int(v) for v in shape.split(","))
        conv = nn.Conv2d(cin, cout, k, s, p, bias=False).to(dev).to(memory_format=torch.channels_last)
        x = torch.randn(a.batch, cin, h, h, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        hip.ensure_channels_last_weight(conv)
        g = hip.conv_geom(x, conv)
        y = hip.conv_forward_raw(x, conv.weight, g)
        dy = torch.randn_like(y)
        flops = 2.0 * g.N * g.OH * g.OW * cout * g.T * cin
        for op in a.ops.split(","):
            run = (lambda: hip.conv_forward_raw(x, conv.weight, g)) if op == "fwd" else \
                (lambda: hip.conv_dgrad_raw(dy, conv.weight, g))
            arms = {"tuned": ("tuned", None)}
            for v, (tm, bn, wm, wn, var) in enumerate(hip.conv_deep_cfgs()):
                if not var & 6:
                    arms[f"deep{v}:{tm}x{bn}/{var}"] = ("deep", v)

            def set_arm(kind, v):
                hip._STAGES_TUNED.clear()
                hip.DEEP_FORCE = v if kind == "deep" else None
                hip.DEEP_CONV = False  # the tuned arm: the pre-existing candidates only

            times = {name: [] for name in arms}
            for name, (kind, v) in arms.items():  # tune each arm once (kernel choice cached per arm below)
                set_arm(kind, v)
                run()
                arms[name] = (kind, v, dict(hip._STAGES_TUNED))
            for _ in range(a.rounds):
                for name, (kind, v, tuned) in arms.items():
                    hip._STAGES_TUNED.clear()
                    hip._STAGES_TUNED.update(tuned)
                    hip.DEEP_FORCE = v if kind == "deep" else None
                    for _ in range(2):
                        run()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        run()
                    e1.record()
                    torch.cuda.synchronize()
                    times[name].append(e0.elapsed_time(e1) / a.iters * 1e3)
            hip.DEEP_FORCE = None
            base = statistics.median(times["tuned"])
            line = f"{op:5s} {shape:18s} b{a.batch}: tuned {base:7.1f} us ({flops / base / 1e6:5.0f} TF)"
            for name in arms:
                if name != "tuned":
                    t = statistics.median(times[name])
                    line += f" | {name} {t:7.1f} ({base / t:4.2f}x)"
            print(line, flush=True)


if __name__ == "__main__":
    main()
