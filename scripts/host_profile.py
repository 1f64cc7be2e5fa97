"""Host (Python) cost of one training step: cProfile over a few steady-state steps of bench's trainer.

    python scripts/host_profile.py [model=inceptionv3] [image=299] [batch=128]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pytorch_imageclassification_distributed_amd.data import DeviceSyntheticLoader
from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser
from pytorch_imageclassification_distributed_amd.parallel import init_distributed

model = sys.argv[1] if len(sys.argv) > 1 else "inceptionv3"
size = int(sys.argv[2]) if len(sys.argv) > 2 else 299
B = int(sys.argv[3]) if len(sys.argv) > 3 else 128
ctx = init_distributed(device="cuda")
targs = build_parser().parse_args(["--synthetic", "--model", model, "--image-size", str(size), "--batchsize", str(B),
                                   "--num-classes", "7", "--num-workers", "0", "--synthetic-train-size", "8",
                                   "--synthetic-val-size", "8", "--no-sync-bn", "--lr", "1e-4"])
tr = Trainer(targs, ctx)
tr.net.train()
batches = list(iter(DeviceSyntheticLoader(B, 7, size, ctx.device, steps=2, ring=2, seed=1)))
for i in range(6):
    tr.train_step(batches[i % 2]["image"], batches[i % 2]["label"])
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for i in range(5):
    tr.train_step(batches[i % 2]["image"], batches[i % 2]["label"])
pr.disable()
torch.cuda.synchronize()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(28)
