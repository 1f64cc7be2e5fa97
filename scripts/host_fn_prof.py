"""Host time per op-layer function (forward AND the autograd engine thread's backward), by wrapping the
functions of ops/hip.py and the _C launchers with perf_counter timers (cProfile sees only the main thread).

    python scripts/host_fn_prof.py MODEL SIZE BATCH
"""
import collections
import functools
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pytorch_imageclassification_distributed_amd.data import DeviceSyntheticLoader
from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser
from pytorch_imageclassification_distributed_amd.ops import hip
from pytorch_imageclassification_distributed_amd.parallel import init_distributed

MODEL = sys.argv[1] if len(sys.argv) > 1 else "inceptionv3"
SIZE = int(sys.argv[2]) if len(sys.argv) > 2 else 299
B = int(sys.argv[3]) if len(sys.argv) > 3 else 128
ctx = init_distributed(device="cuda")
tr = Trainer(build_parser().parse_args(["--synthetic", "--model", MODEL, "--image-size", str(SIZE), "--batchsize", str(B),
                                        "--num-classes", "7", "--num-workers", "0", "--synthetic-train-size", "8",
                                        "--synthetic-val-size", "8", "--no-sync-bn", "--lr", "1e-4"]), ctx)
tr.net.train()
data = list(iter(DeviceSyntheticLoader(B, 7, SIZE, ctx.device, steps=4, ring=2, seed=1)))
for i in range(6):
    tr.train_step(data[i % 4]["image"], data[i % 4]["label"])
torch.cuda.synchronize()

TOT = collections.defaultdict(float)
CNT = collections.defaultdict(int)
local = threading.local()


def wrap(owner, name, label):
    fn = getattr(owner, name)

    @functools.wraps(fn)
    def w(*a, **k):
        depth = getattr(local, "d", 0)
        local.d = depth + 1
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            TOT[(depth, label)] += time.perf_counter() - t
            CNT[(depth, label)] += 1
            local.d = depth
    setattr(owner, name, w)


for cls in ("ConvFn", "BNActFn", "BNActPoolFn", "MaxPoolFn", "AvgPoolFn", "GapFn", "MlpFn", "CrossEntropyFn", "CatFn",
            "DropoutFn", "DwConvFn", "SEFn", "AddFn", "SiblingConvFn", "SiblingBNFn"):
    c = getattr(hip, cls, None)
    if c is not None:
        wrap(c, "forward", f"{cls}.forward")
        wrap(c, "backward", f"{cls}.backward")
for fn in ("conv_forward_raw", "conv_dgrad_raw", "conv_wgrad_raw", "_conv_gemm", "_on_side", "_bn_coef", "_bn_bwd_k",
           "_wgrad_plan", "_wgrad_launch", "weight_bf16", "weight_bf16_t", "_dgrad_phases", "_fwd_taps", "arena_slot",
           "grad_buffer", "_empty_cl", "stat_groups", "conv_bn_act"):
    if hasattr(hip, fn):
        wrap(hip, fn, fn)
for fn in ("conv_gemm", "conv_wgrad", "bn_apply", "bn_bwd_elemt", "bn_bwd_reduce", "bn_reduce_finalize",
           "bn_reduce_bwd", "direct_conv", "bn_fin_apply", "bn_fin_bwd"):
    if hasattr(hip.C, fn):
        wrap(hip.C, fn, "C." + fn)

N = 5
t0 = time.perf_counter()
for i in range(N):
    tr.train_step(data[i % 4]["image"], data[i % 4]["label"])
host = (time.perf_counter() - t0) / N
torch.cuda.synchronize()
print(f"host {host * 1e3:.2f} ms per step ({MODEL} b{B}); per-step time by function (depth, inclusive):")
for (d, k), v in sorted(TOT.items(), key=lambda kv: -kv[1]):
    print(f"  d{d} {k:28s} {v / N * 1e3:7.3f} ms  {CNT[(d, k)] // N:5d} calls  {v / max(CNT[(d, k)], 1) * 1e6:6.1f} us/call")
