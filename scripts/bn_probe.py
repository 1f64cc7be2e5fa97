"""bn_apply (+ residual, ReLU mask) and the BN-backward elementwise pass against torch's add on the same bytes.

    python scripts/bn_probe.py [rows=3211264] [C=256]

ResNet-50 layer1's residual BN at b1024 by default (3.2 M pixels x 256 channels)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 3211264
C = int(sys.argv[2]) if len(sys.argv) > 2 else 256
from pytorch_imageclassification_distributed_amd.ops import hip  # noqa: E402

dev = torch.device("cuda")
y = torch.randn(rows * C, device=dev, dtype=torch.bfloat16)
res = torch.randn(rows * C, device=dev, dtype=torch.bfloat16)
out = torch.empty_like(y)
coef = torch.randn(4 * C, device=dev)
mask = torch.empty(rows * C // 8, device=dev, dtype=torch.uint8)


def t(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


n = rows * C
for name, fn, nb in [
        ("torch add (r2w1)", lambda: torch.add(y, res, out=out), 6 * n),
        ("bn_apply +res +relu +mask", lambda: hip.C.bn_apply(y, coef, res, out, rows, C, C, 0, 1, None, None, mask=mask),
         6 * n + n // 8),
        ("bn_apply +res +relu", lambda: hip.C.bn_apply(y, coef, res, out, rows, C, C, 0, 1, None, None), 6 * n),
        ("bn_apply relu (r1w1)", lambda: hip.C.bn_apply(y, coef, None, out, rows, C, C, 0, 1, None, None), 4 * n),
        ("torch copy (r1w1)", lambda: out.copy_(y), 4 * n)]:
    us = t(fn)
    print(f"{name:28s} rows={rows} C={C}: {us:8.1f} us  {nb / us / 1e6:5.2f} TB/s", flush=True)
