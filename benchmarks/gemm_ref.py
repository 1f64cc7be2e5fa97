"""Our implicit-GEMM kernel on plain GEMMs (1x1 convolutions) against hipBLASLt (torch.mm) on the same
M x N x K, random bf16 operands - a measured ceiling for the conv kernels' main loop.

Rows: the ResNet-50 1x1 forward GEMMs at batch B (M = B*H*W pixels, N = Cout, K = Cin), plus square
GEMMs.  For every row our kernel runs every configuration of the table (best reported, all with
--all) with no BatchNorm epilogue; hipBLASLt computes C[M,N] = A[M,K] @ B[N,K]^T.

    python benchmarks/gemm_ref.py [--batch 512] [--all]
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # (M per image, N, K) of the ResNet-50 1x1 forward GEMMs
    (3136, 256, 64), (3136, 64, 256), (784, 512, 128), (784, 128, 512), (196, 1024, 256),
    (196, 256, 1024), (49, 2048, 512), (49, 512, 2048),
]


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(3):
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--all", action="store_true")
    ap.add_argument("--square", default="4096,8192")
    a = ap.parse_args()
    from pytorch_imageclassification_distributed_amd.ops import hip
    dev = "cuda"
    torch.manual_seed(0)
    rows = [(m * a.batch, n, k) for m, n, k in SHAPES] + [(s, s, s) for s in map(int, a.square.split(",")) if s]
    cfgs = hip.conv_cfgs()
    for (M, N, K) in rows:
        A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
        flop = 2.0 * M * N * K
        t_ref = timeit(lambda: torch.mm(A, B.t()))
        # the conv view of the same GEMM: x = [1, K, M, 1] NHWC == A, 1x1 weight [N, K] == B
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        geo = (M, N, K, K, M, 1, M, 1, 1, K, M, 1, 1, 0, 0, N, 0)
        zero = hip.ws(torch.device(dev)).zero
        res = {}
        for i, (tm, bn, wm, wn, st) in enumerate(cfgs):
            if bn > 64 and bn >= 2 * N:
                continue
            res[f"{tm}x{bn}/{wm}x{wn}/s{st}#{i}"] = timeit(
                lambda: hip.C.conv_gemm(A, B.view(-1), out, None, None, *geo, [0], [0], [0], hip.G_STATS, zero,
                                        None, None, None, None, None, 0, 1, 0, 0, i, None, None, None, None, None, None, None, 0, None, None, None, None, 0))
        for v, (tm, bn, wm, wn, var) in enumerate(hip.conv_deep_cfgs()):
            if (bn > 64 and bn >= 2 * N) or var & 6:
                continue
            res[f"{tm}x{bn}/{wm}x{wn}/deep#{v}"] = timeit(
                lambda: hip.C.conv_gemm(A, B.view(-1), out, None, None, *geo, [0], [0], [0], hip.G_STATS, zero,
                                        None, None, None, None, None, 0, 1, 0, 0, hip.DEEP_BASE + v, None, None, None, None, None, None, None, 0, None, None, None, None, 0))
        ref = torch.mm(A, B.t())
        err = ((out.float() - ref.float()).abs().max() / ref.float().abs().max()).item()  # (last config run)
        best = min(res, key=res.get)
        line = (f"M={M:8d} N={N:5d} K={K:5d}: hipBLASLt {t_ref * 1e3:8.1f}us {flop / t_ref / 1e9:6.0f}TF | "
                f"ours {best:>16} {res[best] * 1e3:8.1f}us {flop / res[best] / 1e9:6.0f}TF (err {err:.1e})")
        print(line, flush=True)
        if a.all:
            print("      " + "  ".join(f"{k}:{flop / v / 1e9:.0f}" for k, v in sorted(res.items(), key=lambda kv: kv[1])),
                  flush=True)


if __name__ == "__main__":
    main()
