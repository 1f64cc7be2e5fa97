"""Per-candidate weight-gradient timings (split target x kernel variant) for the narrow-Cout ResNet-50
layers at batch 512, from the tuner's own timing loop (ops/hip.py _wgrad_config -> WGRAD_TUNE_LOG).
Variants (at the time of profiles/history/r4d_wgrad_wide_tiles_probe.txt): 1 / 2 = 64|128 x 128 tile, 1- / 2-stage
ring, 3 = 8-wave in-block pixel split,
8 = 4-deep ring of 32-pixel stages, 10 / 11 = 64 x 256, 12 / 13 = 128 x 256."""
import sys

import torch
import torch.nn as nn

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from pytorch_imageclassification_distributed_amd.ops import hip  # noqa: E402

CL = torch.channels_last
SHAPES = [  # N, Cin, H, W, Cout, k, stride, pad
    (512, 16, 113, 113, 64, (4, 4), 1, (1, 1)),   # ~ the space-to-depth stem
    (512, 64, 56, 56, 64, (3, 3), 1, (1, 1)),
    (512, 256, 56, 56, 64, (1, 1), 1, (0, 0)),
    (512, 128, 28, 28, 128, (3, 3), 1, (1, 1)),
    (512, 512, 28, 28, 128, (1, 1), 1, (0, 0)),
    (512, 256, 56, 56, 128, (1, 1), 1, (0, 0)),
]
for n, cin, h, w, cout, k, s, p in SHAPES:
    conv = nn.Conv2d(cin, cout, k, s, p, bias=False).cuda().to(memory_format=CL)
    x = torch.randn(n, cin, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=CL)
    y = hip.ConvFn.apply(x, conv.weight, conv, False)
    hip.WGRAD_TUNE_LOG.clear()
    y.backward(torch.randn_like(y))
    torch.cuda.synchronize()
    for co, ntot, m, times in hip.WGRAD_TUNE_LOG:
        best = min(times, key=times.get)
        print(f"Cout={co} Ntot={ntot} M={m}: best {best} {times[best] * 1e3:.1f} us", flush=True)
        by_var = {}
        for (cand, st), t in times.items():
            by_var.setdefault(st, []).append((t, cand))
        for st in sorted(by_var):
            t, cand = min(by_var[st])
            print(f"   variant {st:2d}: {t * 1e3:7.1f} us (split target {cand})", flush=True)
