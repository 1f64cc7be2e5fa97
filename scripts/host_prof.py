"""Host-side (CPU) profile of the training step: where does enqueue time go?"""
import cProfile
import pstats
import sys
import time

import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

sys.argv = [sys.argv[0]] + sys.argv[1:]
from pytorch_imageclassification_distributed_amd.data import DeviceSyntheticLoader
from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser
from pytorch_imageclassification_distributed_amd.parallel import init_distributed

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
MODEL = sys.argv[2] if len(sys.argv) > 2 else "resnet50"
SIZE = int(sys.argv[3]) if len(sys.argv) > 3 else 224
ctx = init_distributed(device="cuda")
targs = build_parser().parse_args(["--synthetic", "--model", MODEL, "--image-size", str(SIZE), "--batchsize", str(B),
                                   "--num-classes", "7",
                                   "--num-workers", "0", "--synthetic-train-size", "8", "--synthetic-val-size", "8",
                                   "--no-sync-bn", "--lr", "1e-4"])
tr = Trainer(targs, ctx)
tr.net.train()
batches = list(iter(DeviceSyntheticLoader(B, 7, SIZE, ctx.device, steps=4, ring=2, seed=1)))
for i in range(8):
    tr.train_step(batches[i % 4]["image"], batches[i % 4]["label"])
torch.cuda.synchronize()
for n in range(3):
    t = time.perf_counter(); tr.train_step(batches[0]["image"], batches[0]["label"]); th = time.perf_counter() - t
    torch.cuda.synchronize(); tt = time.perf_counter() - t
    print(f"host {th*1e3:.1f} ms  total {tt*1e3:.1f} ms")
pr = cProfile.Profile()
pr.enable()
for i in range(5):
    tr.train_step(batches[i % 4]["image"], batches[i % 4]["label"])
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(45)
st.sort_stats("cumulative").print_stats(40)
