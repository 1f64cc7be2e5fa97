import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pytorch_imageclassification_distributed_amd.data import DeviceSyntheticLoader
from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser
from pytorch_imageclassification_distributed_amd.ops import hip
from pytorch_imageclassification_distributed_amd.parallel import init_distributed
ctx = init_distributed(device="cuda")
B = 128
targs = build_parser().parse_args(["--synthetic", "--model", "inceptionv3", "--image-size", "299", "--batchsize", str(B), "--num-classes", "7",
                                   "--num-workers", "0", "--synthetic-train-size", "8", "--synthetic-val-size", "8", "--no-sync-bn", "--lr", "1e-4"])
tr = Trainer(targs, ctx)
tr.net.train()
batches = list(iter(DeviceSyntheticLoader(B, 7, 299, ctx.device, steps=2, ring=2, seed=1)))
for i in range(6):
    tr.train_step(batches[i % 2]["image"], batches[i % 2]["label"])
torch.cuda.synchronize()
for k, v in hip._STAGES_TUNED.items():
    if v[2] >= hip.DIRECT_BASE:
        print("direct", v[2] - hip.DIRECT_BASE, "geo", k[0][:8], "bwd-link", k[7])
for (m, n, kk, times) in hip.TUNE_LOG:
    d = {c: t for c, t in times.items() if c[2] >= hip.DIRECT_BASE}
    if d:
        best = min(times, key=times.get)
        print(m, n, kk, "best", best, f"{times[best]*1e3:.0f}us", {c[2]: round(t * 1e3) for c, t in d.items()})
t0 = time.time()
for i in range(10):
    tr.train_step(batches[i % 2]["image"], batches[i % 2]["label"])
torch.cuda.synchronize()
print("ms/step", (time.time() - t0) * 100)
