"""Whole-step HIP graph vs eager: identical inputs and initial weights, step-by-step losses and final
parameters.  Deterministic mode (--det): every kernel is order-deterministic, so the graph must match
eager bitwise; default mode: losses must track.

    python scripts/graph_check.py --model resnet50 --batch 64 --steps 12 [--det]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from pytorch_imageclassification_distributed_amd.data import DeviceSyntheticLoader
from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser
from pytorch_imageclassification_distributed_amd.parallel import init_distributed

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="resnet50")
ap.add_argument("--image-size", type=int, default=224)
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--steps", type=int, default=12)
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--det", action="store_true")
a = ap.parse_args()
ctx = init_distributed(device="cuda")


def make():
    args = ["--synthetic", "--model", a.model, "--image-size", str(a.image_size), "--batchsize", str(a.batch),
            "--num-classes", "7", "--num-workers", "0", "--synthetic-train-size", "8", "--synthetic-val-size", "8",
            "--no-sync-bn", "--lr", "1e-4", "--seed", "5"] + (["--deterministic"] if a.det else [])
    tr = Trainer(build_parser().parse_args(args), ctx)
    tr.net.train()
    return tr


data = list(iter(DeviceSyntheticLoader(a.batch, 7, a.image_size, ctx.device, steps=a.steps, ring=2, seed=11)))
eager = make()
le = [float(eager.train_step(d["image"], d["label"]).item()) for d in data]
pe = [p.detach().clone() for p in eager.model.parameters()]
bufe = [b.detach().clone() for b in eager.model.buffers()]
del eager
torch.cuda.synchronize()
graph = make()
lg = []
for i, d in enumerate(data):
    if i < a.warmup:
        lg.append(float(graph.train_step(d["image"], d["label"]).item()))
    else:
        lg.append(float(graph.graph_step(d["image"], d["label"]).item()))
torch.cuda.synchronize()
pg = [p.detach() for p in graph.model.parameters()]
bufg = [b.detach() for b in graph.model.buffers()]
for i, (x, y) in enumerate(zip(le, lg)):
    print(f"step {i:2d} eager {x:.6f} graph {y:.6f} {'(graph)' if i >= a.warmup else ''} {'SAME' if x == y else 'DIFF'}")
dp = max((x.float() - y.float()).abs().max().item() for x, y in zip(pe, pg))
db = max((x.float() - y.float()).abs().max().item() for x, y in zip(bufe, bufg))
same = all(torch.equal(x, y) for x, y in zip(pe, pg)) and all(torch.equal(x, y) for x, y in zip(bufe, bufg))
print(f"max |param diff| {dp:.3e}  max |buffer diff| {db:.3e}  bitwise equal: {same}")
if a.det and not same:
    sys.exit(1)
