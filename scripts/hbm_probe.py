"""Practical HBM bandwidth of simple streams on this GPU (the yardstick for the elementwise kernels).

    python scripts/hbm_probe.py [GB=1.6]

Times torch's own vectorised kernels on bf16 tensors of the given size: copy (read 1 + write 1), add (read 2 +
write 1), a read-only sum, and a zero fill (write only), and prints the achieved TB/s of each."""
import sys

import torch

GB = float(sys.argv[1]) if len(sys.argv) > 1 else 1.6
n = int(GB * 1e9 / 2)
dev = torch.device("cuda")
a = torch.randn(n, device=dev, dtype=torch.bfloat16)
b = torch.randn(n, device=dev, dtype=torch.bfloat16)
o = torch.empty_like(a)


def t(fn, nbytes, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return ms, nbytes / ms / 1e9


for name, fn, nb in [("copy  r1w1", lambda: o.copy_(a), 4 * n), ("add   r2w1", lambda: torch.add(a, b, out=o), 6 * n),
                     ("sum   r1  ", lambda: a.sum(dtype=torch.float32), 2 * n), ("fill  w1  ", lambda: o.zero_(), 2 * n)]:
    ms, tbs = t(fn, nb)
    print(f"{name} {GB:.1f} GB tensors: {ms * 1e3:8.1f} us  {tbs:5.2f} TB/s", flush=True)
