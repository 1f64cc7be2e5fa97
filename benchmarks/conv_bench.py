"""Per-shape conv kernel benchmark: our MFMA implicit-GEMM (fwd / dgrad / wgrad) vs MIOpen.

Shapes: the 23 unique ResNet-50 @224 convolutions at a given batch.
Prints one line per shape and a JSON summary (TFLOP/s = 2*MACs / time).

    python benchmarks/conv_bench.py --batch 256 [--torch]
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# Cin, Cout, k, s, p, H_in, count   (ResNet-50 @224)
R50 = [
    (256, 256, 3, 1, 1, 14, 5), (64, 64, 3, 1, 1, 56, 3), (128, 128, 3, 1, 1, 28, 3),
    (256, 1024, 1, 1, 0, 14, 6), (1024, 256, 1, 1, 0, 14, 5), (512, 512, 3, 1, 1, 7, 2),
    (64, 256, 1, 1, 0, 56, 4), (128, 512, 1, 1, 0, 28, 4), (512, 128, 1, 1, 0, 28, 3),
    (512, 2048, 1, 1, 0, 7, 3), (8, 64, 7, 2, 3, 224, 1), (128, 128, 3, 2, 1, 56, 1),
    (256, 256, 3, 2, 1, 28, 1), (512, 512, 3, 2, 1, 14, 1), (256, 64, 1, 1, 0, 56, 2),
    (256, 128, 1, 1, 0, 56, 1), (256, 512, 1, 2, 0, 56, 1), (512, 256, 1, 1, 0, 28, 1),
    (512, 1024, 1, 2, 0, 28, 1), (1024, 512, 1, 1, 0, 14, 1), (1024, 2048, 1, 2, 0, 14, 1),
    (2048, 512, 1, 1, 0, 7, 2), (64, 64, 1, 1, 0, 56, 1),
]


def timeit(fn, iters=10, warm=2):
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / iters


def _cfg_name(hip, c):
    if c[2] < 0:
        return f"st{c[0]}/n{c[1]}"
    if c[2] >= hip.DIRECT_BASE:
        cip, cot = hip.DIRECT_CFGS[c[2] - hip.DIRECT_BASE]
        return f"direct{cip}/{cot}"
    tm, bn, wm, wn, st = hip.conv_cfgs()[c[2]]
    return f"{tm}x{bn}/{wm}x{wn}/s{st}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--torch", action="store_true", help="also time MIOpen (torch) for each shape")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default="", help="comma list of conv fwd/dgrad kernel variants to A/B (1,2,3)")
    ap.add_argument("--single", default="", help="comma list of 1-stage-ring k-step thresholds to A/B (0 = never)")
    ap.add_argument("--wvariants", default="", help="comma list of wgrad kernel variants to A/B (1,2)")
    ap.add_argument("--wblocks", default="", help="comma list of wgrad split-K target block counts to sweep")
    ap.add_argument("--tune-log", action="store_true", help="print every fwd/dgrad tuning candidate's time")
    ap.add_argument("--only", default="", help="comma list of shape indices (into R50) to run")
    a = ap.parse_args()
    from pytorch_imageclassification_distributed_amd.ops import hip
    dev = "cuda"
    n = a.batch
    rows = []
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0, "t_fwd": 0.0, "t_bwd": 0.0}
    shapes = [R50[int(i)] for i in a.only.split(",")] if a.only else R50
    for (ci, co, k, s, p, h, cnt) in shapes:
        hip.TUNE_LOG.clear()
        hip.WGRAD_TUNE_LOG.clear()
        conv = nn.Conv2d(ci, co, k, s, p, bias=False).to(dev).to(memory_format=torch.channels_last)
        x = torch.randn(n, ci, h, h, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        g = hip.ConvGeom(x, conv)
        stats = hip.ws(x.device).stats_buf(co)
        part_sums = torch.empty(2 * co, dtype=torch.float64, device=dev)
        y = hip.conv_forward_raw(x, conv.weight, g, stats=stats)
        hip.C.bn_partials(stats, hip.G_STATS, co, part_sums, None, None)
        dy = torch.randn_like(y)
        macs = n * g.OH * g.OW * co * ci * k * k
        tf = lambda ms: 2 * macs / (ms * 1e-3) / 1e12  # noqa: E731

        def fwd():
            hip.conv_forward_raw(x, conv.weight, g, stats=stats)
            hip.C.bn_partials(stats, hip.G_STATS, co, part_sums, None, None)

        if a.variants:
            alt = []
            for v in [int(t) for t in a.variants.split(",")]:
                hip.C.conv_set_variant(v)
                alt.append((v, timeit(fwd, a.iters), timeit(lambda: hip.conv_dgrad_raw(dy, conv.weight, g), a.iters)
                            if ci != 8 else 0.0))
            hip.C.conv_set_variant(0)
            print("   variants " + "  ".join(f"v{v}: fwd {tf_:.3f} dgrad {td_:.3f}" for v, tf_, td_ in alt), flush=True)
        if a.single:
            alt, keep = [], hip.CONV_STAGES
            hip.CONV_STAGES = "0"
            for nk in [int(t) for t in a.single.split(",")]:
                hip.C.conv_set_single_stage(nk)
                alt.append((nk, timeit(fwd, a.iters), timeit(lambda: hip.conv_dgrad_raw(dy, conv.weight, g), a.iters)
                            if ci != 8 else 0.0))
            hip.C.conv_set_single_stage(4)
            hip.CONV_STAGES = keep
            print("   single-stage " + "  ".join(f"nk<={v}: fwd {tf_:.3f} dgrad {td_:.3f}" for v, tf_, td_ in alt),
                  flush=True)
        if a.wvariants:
            alt = []
            for v in [int(t) for t in a.wvariants.split(",")]:
                hip.C.conv_set_wgrad_variant(v)
                alt.append((v, timeit(lambda: hip.conv_wgrad_raw(dy, x, conv.weight, g), a.iters)))
            hip.C.conv_set_wgrad_variant(0)
            print("   wgrad variants " + "  ".join(f"w{v}: {t:.3f}" for v, t in alt), flush=True)
        if a.wblocks:
            alt, keep = [], hip.WGRAD_TARGET_BLOCKS
            for nb in [int(t) for t in a.wblocks.split(",")]:
                hip.WGRAD_TARGET_BLOCKS = nb
                alt.append((nb, timeit(lambda: hip.conv_wgrad_raw(dy, x, conv.weight, g), a.iters)))
            hip.WGRAD_TARGET_BLOCKS = keep
            print("   wgrad blocks " + "  ".join(f"{nb}: {t:.3f}" for nb, t in alt), flush=True)
        t_f = timeit(fwd, a.iters)
        t_d = timeit(lambda: hip.conv_dgrad_raw(dy, conv.weight, g), a.iters) if ci != 8 else 0.0
        t_w = timeit(lambda: hip.conv_wgrad_raw(dy, x, conv.weight, g), a.iters)
        r = dict(shape=f"{ci}->{co} k{k}s{s} {h}x{h}", count=cnt, fwd_ms=t_f, dgrad_ms=t_d, wgrad_ms=t_w,
                 fwd_tf=tf(t_f), dgrad_tf=tf(t_d) if t_d else None, wgrad_tf=tf(t_w))
        tot["fwd"] += t_f * cnt
        tot["dgrad"] += t_d * cnt
        tot["wgrad"] += t_w * cnt
        if a.torch:
            xt = x.detach().requires_grad_(True)
            wt = conv.weight.detach().to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
            tt_f = timeit(lambda: F.conv2d(xt, wt, None, s, p), a.iters)
            yt = F.conv2d(xt, wt, None, s, p)
            tt_b = timeit(lambda: torch.autograd.grad(yt, [xt, wt], dy, retain_graph=True), a.iters)
            r.update(torch_fwd_ms=tt_f, torch_bwd_ms=tt_b, torch_fwd_tf=tf(tt_f))
            tot["t_fwd"] += tt_f * cnt
            tot["t_bwd"] += tt_b * cnt
        rows.append(r)
        msg = (f"{r['shape']:>26} x{cnt}: fwd {t_f:7.3f}ms {r['fwd_tf']:6.0f}TF | dgrad {t_d:7.3f}ms "
               f"{(r['dgrad_tf'] or 0):6.0f}TF | wgrad {t_w:7.3f}ms {r['wgrad_tf']:6.0f}TF")
        if a.torch:
            msg += f" || miopen fwd {r['torch_fwd_ms']:7.3f}ms bwd {r['torch_bwd_ms']:7.3f}ms"
        print(msg, flush=True)
        if a.tune_log:
            for (m_, n_, k_, times) in hip.TUNE_LOG:
                best = min(times, key=times.get)
                print(f"      tune M={m_} N={n_} K={k_}: " + "  ".join(
                    f"{'*' if c == best else ''}{_cfg_name(hip, c)}:{t * 1e3:.0f}us" for c, t in times.items()),
                    flush=True)
            for (co_, nt_, m_, times) in hip.WGRAD_TUNE_LOG:
                best = min(times, key=times.get)
                print(f"      wgrad Co={co_} Ntot={nt_} pix={m_}: " + "  ".join(
                    f"{'*' if c == best else ''}b{c[0]}/st{c[1]}:{t * 1e3:.0f}us" for c, t in times.items()),
                    flush=True)
    print("tuned wgrad (blocks, stages):", {f"{k[4]}<-{k[1]} k{k[5]}s{k[7]} {k[2]}x{k[3]}": v
                                             for k, v in hip._WGRAD_TUNED.items()})
    print("tuned fwd/dgrad configs:", sorted(collections.Counter(_cfg_name(hip, c) for c in hip._STAGES_TUNED.values()).items()))
    print(json.dumps({"batch": n, "total_ms": tot, "rows": rows}))


if __name__ == "__main__":
    main()
