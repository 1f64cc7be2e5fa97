"""Run ONE plain GEMM C[M,N] = A[M,K] B[N,K]^T repeatedly with one kernel (for rocprofv3 --pmc passes).

    python scripts/gemm_probe.py --mnk 8192,8192,8192 --kernel deep0|cfg11|blas [--iters 20]

``deepV``: entry V of ops.hip.conv_deep_cfgs(); ``cfgI``: entry I of ops.hip.conv_cfgs(); ``blas``: torch.mm
(hipBLASLt).  The conv kernels run the 1x1 "GEMM view" of benchmarks/gemm_ref.py.  Random [-1, 1) bf16 data.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mnk", default="8192,8192,8192")
    ap.add_argument("--kernel", default="deep0")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--check", action="store_true", help="compare with an fp32 reference (an extra GEMM launch)")
    a = ap.parse_args()
    from pytorch_imageclassification_distributed_amd.ops import hip
    M, N, K = (int(v) for v in a.mnk.split(","))
    dev = "cuda"
    torch.manual_seed(0)
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    geo = (M, N, K, K, M, 1, M, 1, 1, K, M, 1, 1, 0, 0, N, 0)
    zero = hip.ws(torch.device(dev)).zero
    if a.kernel == "blas":
        run = lambda: torch.mm(A, B.t(), out=out)  # noqa: E731
    else:
        cfg = hip.DEEP_BASE + int(a.kernel[4:]) if a.kernel.startswith("deep") else int(a.kernel[3:])
        run = lambda: hip.C.conv_gemm(A, B.view(-1), out, None, None, *geo, [0], [0], [0], hip.G_STATS, zero,  # noqa: E731
                                      None, None, None, None, None, 0, 1, 0, 0, cfg, None, None, None, None, None,
                                      None, None, 0, None, None, None, None, 0)
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
    err = float("nan")
    if a.check:
        ref = A.float() @ B.float().t()
        err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
    print(f"{a.kernel} M={M} N={N} K={K}: {ms * 1e3:.1f} us  {2.0 * M * N * K / ms / 1e9:.0f} TF/s  (err {err:.1e})",
          flush=True)


if __name__ == "__main__":
    main()
