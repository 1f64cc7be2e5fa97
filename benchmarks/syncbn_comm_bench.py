"""Latency of the SyncBN statistics exchange: one-shot peer kernel (parallel/peer.py) vs torch.distributed.

usage (one rank per GPU on a multi-GPU node, RCCL for the comparison):
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/syncbn_comm_bench.py
on a 1-GPU box (ranks share the GPU; torch.distributed = gloo, so only the peer column is meaningful):
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 benchmarks/syncbn_comm_bench.py --backend gloo

Each size is the fp64 payload of one ResNet-50 BN layer (2C+1 forward, 2C backward); calls are issued
back to back on one stream, as in a training step, and timed with HIP events.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pytorch_imageclassification_distributed_amd.parallel import init_distributed  # noqa: E402
from pytorch_imageclassification_distributed_amd.parallel import peer  # noqa: E402


def timed(fn, t, iters):
    for _ in range(10):
        fn(t)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn(t)
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--backend", default="auto")
    p.add_argument("--iters", type=int, default=500)
    a = p.parse_args()
    ctx = init_distributed(device="cuda", backend=a.backend)
    grp = dist.new_group(list(range(ctx.world_size)))
    assert peer.setup_peer_syncbn(grp, ctx.device, "peer")
    rows = []
    for c in (64, 256, 1024, 2048):
        n = 2 * c + 1
        t = torch.randn(n, dtype=torch.float64, device=ctx.device)
        us_peer = timed(lambda x: peer.stats_all_reduce_(x, grp), t, a.iters)
        us_dist = timed(lambda x: dist.all_reduce(x, group=grp), t, max(a.iters // 5, 20))
        rows.append({"C": c, "elems": n, "peer_us": round(us_peer, 2), f"{ctx.backend}_us": round(us_dist, 2)})
    assert peer.peer_errors() == 0
    if ctx.rank == 0:
        for r in rows:
            print(json.dumps({"world": ctx.world_size, **r}), flush=True)
    peer.teardown_peer_syncbn()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
