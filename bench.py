"""Headline benchmark: images/sec (whole node), ResNet-50 224x224 bf16, DDP over N MI355X.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it
is launched by ``torch.distributed.run`` with one rank per GPU (RCCL over xGMI).
W untimed warmup steps, then exactly K timed steps bracketed by a barrier and
``torch.cuda.synchronize()``; the max time over ranks is reported; rank 0
prints ONE JSON line.

Workload per step = the reference training step (reference train.py:44-73):
forward (ResNet-50 + reference MLP head, 7 classes, class-weighted CE), loss
all-reduce / world, backward with bucketed gradient all-reduce overlapped, Adam
step.  Synthetic data (fp32 NCHW normalised images generated on device,
converted to bf16 NHWC inside the step), random-init weights, per-GPU batch
fixed (weak scaling).  SyncBN follows the reference semantics (on when N>1).

``--compute torch`` runs the *reference stack* (torch DDP + nn.SyncBatchNorm +
bf16 autocast over ATen/MIOpen) on the identical workload for the baseline.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import torch
import torch.distributed as dist

from pytorch_imageclassification_distributed_amd.data import DeviceSyntheticLoader, HostSyntheticLoader
from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser
from pytorch_imageclassification_distributed_amd.engine.config import GRAPH_AUTO_MAX_BATCH
from pytorch_imageclassification_distributed_amd.parallel import barrier, destroy, init_distributed

HERE = os.path.dirname(os.path.abspath(__file__))
METRIC = "images/sec (whole node) ResNet-50 224x224 bf16 at 1/2/4/8 MI355X"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=10)
    # 1024 per GPU (44 GiB of the 288 GB HBM3E): +4-5 % img/s over 512 on one GPU (fuller last waves on the
    # 14x14 / 7x7 layers, per-step fixed costs amortised; profiles/history/r4g_b1024_tuning_runs.txt) and half the
    # share of per-step SyncBN / all-reduce latency at N>1; the reference stack is measured at the same
    # batch (benchmarks/reference_stack.json)
    p.add_argument("--batch", type=int, default=1024, help="per-GPU batch")
    p.add_argument("--model", default="resnet50")
    p.add_argument("--image-size", type=int, default=224)
    p.add_argument("--num-classes", type=int, default=7)
    p.add_argument("--compute", default="hip", choices=["hip", "torch"])
    p.add_argument("--sync-bn", default="auto", choices=["auto", "on", "off"])
    p.add_argument("--bucket-mb", type=float, default=32.0)
    p.add_argument("--tail-bucket-mb", type=float, default=4.0,
                   help="pieces of the last gradient bucket (stem + layer1, produced last), MiB; 0 = one bucket")
    p.add_argument("--syncbn-comm", default="auto", choices=["auto", "peer", "rccl"],
                   help="SyncBN statistics transport (parallel/peer.py): one-shot xGMI peer kernel or RCCL")
    p.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--comm-backend", default="pg", choices=["pg", "rccl"],
                   help="gradient all-reduce through ProcessGroupNCCL (pg) or the native C++ RCCL communicator")
    p.add_argument("--dist-backend", default="auto", help="auto (RCCL) | gloo (functional multi-rank runs on one GPU)")
    p.add_argument("--profile-steps", type=int, default=0)
    p.add_argument("--tune-db", default="", help="kernel-choice find-db to seed the per-shape tuner with "
                   "(default: $IMGCLS_TUNE_DB, else tuning/mi355x_find_db.json; 'none' disables); shapes it "
                   "does not list are still timed")
    p.add_argument("--tune-save", default="", help="write the kernel choices of this run to this file")
    p.add_argument("--graph", default="auto", choices=["on", "off", "auto"],
                   help="replay the whole training step as one captured HIP graph (at N > 1: forward + backward, "
                        "then one flat gradient all-reduce and Adam); auto = on "
                        "at per-GPU batch <= 64 (host-bound steps, train.py --hip-graph auto)")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"],
                   help="compute dtype: bf16 (the headline), or fp8 = the experimental MX-FP8 forward convolutions "
                        "(e4m3 operands with block scales, bf16 backward; BASELINE.json config 5).  fp8 measured no "
                        "speed-up over bf16 (README, BASELINE.md), and its JSON line says what ran")
    p.add_argument("--data", default="device", choices=["device", "host"],
                   help="device: batches generated once in HBM (the step alone); host: pinned uint8 host batches "
                        "copied by hipMemcpyAsync on a copy stream and normalised on the GPU inside the timed loop "
                        "(the real-data path minus decode, K24/K25)")
    p.add_argument("--host-input", default="fused", choices=["fused", "fp32"],
                   help="--data host: fused = uint8 -> model input (bf16, s2d stem layout) in one kernel on the copy "
                        "stream; fp32 = the older normalize_u8 to fp32 NCHW, converted again inside the step")
    p.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                   help="cpu: functional rehearsal of the multi-rank path over gloo (no GPU; never a benchmark)")
    p.add_argument("--comm-timing", default="auto", choices=["auto", "on", "off"],
                   help="per-step device-event timeline of the gradient all-reduce (auto: on when N > 1): "
                        "overlap window, side-stream tail and exposed collective time in the JSON line")
    return p.parse_args()


def load_baseline(n_gpus: int, batch: int, model: str = "resnet50", image_size: int = 224):
    """Reference-stack images/sec measured on MI355X for the same model, image size, per-GPU batch and GPU
    count (``images_per_sec`` holds ResNet-50 @224, the headline; ``models`` the others); None if not
    measured."""
    path = os.path.join(HERE, "benchmarks", "reference_stack.json")
    try:
        with open(path) as f:
            ref = json.load(f)
        if model == "resnet50" and image_size == 224:
            table = ref.get("images_per_sec", {})
        else:
            table = ref.get("models", {}).get(f"{model}@{image_size}", {})
        v = table.get(str(batch), {}).get(str(n_gpus))
        return float(v) if v else None
    except (OSError, ValueError, AttributeError):
        return None


def _alloc_counters(dev):
    if dev.type != "cuda":
        return {}
    s = torch.cuda.memory_stats(dev)
    return {"device_malloc": s.get("num_device_alloc", 0), "device_free": s.get("num_device_free", 0),
            "alloc_retries": s.get("num_alloc_retries", 0), "ooms": s.get("num_ooms", 0)}


def _syncbn_checks(tr, ctx) -> dict:
    """SyncBN end-of-run checks across the real GPUs: no peer exchange timed out, and every rank holds
    bitwise the same BN running statistics (each rank sums the same per-rank payloads in rank order, so
    any transport fault - a stale or torn slot - shows up as a mismatch)."""
    from pytorch_imageclassification_distributed_amd.parallel import peer_errors
    out = {"peer_errors": int(peer_errors()) if tr.syncbn_peer else 0}
    bufs = [b.detach().double().reshape(-1) for n, b in tr.model.named_buffers() if "running_" in n]
    if bufs:
        flat = torch.cat(bufs)
        ref = flat.clone()
        dist.broadcast(ref, 0)
        out["syncbn_running_stats_equal_across_ranks"] = bool(torch.equal(ref, flat))
        ok = torch.tensor([1 if out["syncbn_running_stats_equal_across_ranks"] and not out["peer_errors"] else 0],
                          dtype=torch.int32, device=flat.device)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        out["syncbn_running_stats_equal_across_ranks"] = bool(ok.item())
    return out


def _from_slowest_rank(extra: dict, dt: float, ctx, steps: int) -> dict:
    """The diagnostics of the rank whose timed loop took longest (the one the reported time is from), plus
    which rank that was and every rank's own ms/step (a straggler GPU or link shows up here)."""
    box = [None] * ctx.world_size
    dist.all_gather_object(box, (dt, extra))
    slow = max(range(ctx.world_size), key=lambda r: box[r][0])
    return {**box[slow][1], "slowest_rank": slow,
            "rank_ms_per_step": [round(b[0] / steps * 1e3, 3) for b in box]}


def _spawn_ranks(a) -> int:
    """``--gpus N`` without a launcher: start N ranks under torch.distributed.run (one per GPU, rendezvous on
    127.0.0.1) as a child process and return its exit code.  Runs before this process touches the GPU."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] launching {a.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize()


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return _spawn_ranks(a)
    if a.device == "cpu":
        a.compute = "torch"  # the HIP kernels need the GPU; the rehearsal checks launch, rendezvous, reporting
        if a.data == "host":  # the host loader's copy stream and u8 conversion kernel are GPU-only
            print("[bench] --device cpu: --data host needs a GPU copy stream; rehearsing with --data device",
                  file=sys.stderr, flush=True)
            a.data = "device"
    backend = a.dist_backend if a.device == "cuda" else "gloo"
    ctx = init_distributed(device=a.device, backend=backend)
    if ctx.world_size != a.gpus:
        print(f"[bench] world size {ctx.world_size} != --gpus {a.gpus}: refusing to report a mislabelled number",
              file=sys.stderr, flush=True)
        destroy()
        return 2
    sync_bn = (a.sync_bn == "on") or (a.sync_bn == "auto" and ctx.world_size > 1)
    targs = build_parser().parse_args([
        "--synthetic", "--model", a.model, "--image-size", str(a.image_size),
        "--batchsize", str(a.batch), "--num-classes", str(a.num_classes),
        "--num-workers", "0", "--synthetic-train-size", "8", "--synthetic-val-size", "8",
        "--compute", a.compute, "--bucket-mb", str(a.bucket_mb), "--tail-bucket-mb", str(a.tail_bucket_mb), "--comm-dtype", a.comm_dtype, "--comm-backend", a.comm_backend,
        "--lr", "1e-4", "--dtype", a.dtype, "--syncbn-comm", a.syncbn_comm,
    ] + ([] if sync_bn else ["--no-sync-bn"]))
    if ctx.device.type == "cuda":
        free, total = torch.cuda.mem_get_info(ctx.device)
        print(f"[bench] rank {ctx.rank}: device memory {free / 2**30:.1f} GiB free of {total / 2**30:.1f} GiB",
              file=sys.stderr, flush=True)
    tr = Trainer(targs, ctx)
    tr.net.train()
    tune_db = a.tune_db or os.environ.get("IMGCLS_TUNE_DB", "") or os.path.join(HERE, "tuning", "mi355x_find_db.json")
    if a.compute == "hip" and tune_db and tune_db != "none" and os.path.exists(tune_db):
        from pytorch_imageclassification_distributed_amd.ops import hip
        n = hip.load_tuning(tune_db)
        print(f"[bench] rank {ctx.rank}: {n} kernel choices from {tune_db}", file=sys.stderr, flush=True)
    if a.data == "host":
        data = HostSyntheticLoader(a.batch, a.num_classes, a.image_size, ctx.device,
                                   steps=a.warmup + a.steps + 1, ring=2, seed=1234 + ctx.rank)
        if a.host_input == "fused":
            data.input_fn = tr.input_fn  # uint8 -> the model's bf16 input in one kernel on the copy stream
        host_it = iter(data)
    else:
        data = DeviceSyntheticLoader(a.batch, a.num_classes, a.image_size, ctx.device,
                                     steps=a.warmup + a.steps, ring=2, seed=1234 + ctx.rank)
        batches = list(iter(data))

    # at N > 1 the replay holds forward + backward (+ the SyncBN peer exchanges); the gradient all-reduce and
    # Adam follow each replay (Trainer.capture_step)
    use_graph = a.compute == "hip" and tr.graph_capable() and (
        a.graph == "on" or (a.graph == "auto" and a.batch <= GRAPH_AUTO_MAX_BATCH))

    def step(i):
        b = next(host_it) if a.data == "host" else batches[i]
        if use_graph and i >= 2:  # two eager steps tune every kernel shape, then capture / replay
            loss = tr.graph_step(b["image"], b["label"])
        else:
            loss = tr.train_step(b["image"], b["label"])
        return tr.reduce_loss(loss)

    for i in range(a.warmup):
        last = step(i)
    _sync(ctx.device)
    # host enqueue cost of one step (diagnostic, stderr): > ms_per_step would mean CPU-bound
    t_host = time.perf_counter()
    last = step(max(a.warmup - 1, 0))
    t_host = time.perf_counter() - t_host
    _sync(ctx.device)
    print(f"[bench] rank {ctx.rank}: host enqueue {t_host * 1e3:.1f} ms/step", file=sys.stderr, flush=True)
    if a.compute == "hip" and ctx.device.type == "cuda":
        from pytorch_imageclassification_distributed_amd.ops import hip as _h
        # shapes the find-db did not cover were timed during warmup: their picks can differ between processes
        print(f"[bench] rank {ctx.rank}: timed at run time (not in the find-db): {len(_h.TUNE_LOG)} conv, "
              f"{len(_h.WGRAD_TUNE_LOG)} weight-gradient shapes", file=sys.stderr, flush=True)
    if not torch.isfinite(last).item():
        raise FloatingPointError(f"non-finite loss in warmup: {last.item()}")
    comm_t = None
    if ctx.device.type == "cuda" and not use_graph and (
            a.comm_timing == "on" or (a.comm_timing == "auto" and ctx.world_size > 1)):
        from pytorch_imageclassification_distributed_amd.parallel import comm_timer
        comm_t = comm_timer.install()
    barrier(ctx)
    _sync(ctx.device)
    m0 = _alloc_counters(ctx.device)
    t0 = time.perf_counter()
    for i in range(a.steps):
        last = step(a.warmup + i)
    _sync(ctx.device)
    barrier(ctx)
    _sync(ctx.device)
    dt = time.perf_counter() - t0
    if ctx.device.type == "cuda":
        m1 = _alloc_counters(ctx.device)
        # allocator activity inside the timed steps (diagnostic): device mallocs / frees / OOM retries
        # there mean the caching allocator is not in steady state (every hipMalloc / hipFree syncs)
        print(f"[bench] rank {ctx.rank}: peak memory {torch.cuda.max_memory_allocated(ctx.device) / 2**30:.1f} GiB "
              f"(reserved {torch.cuda.max_memory_reserved(ctx.device) / 2**30:.1f} GiB); "
              f"timed-region allocator events: " + ", ".join(f"{k} {m1[k] - m0[k]}" for k in m0),
              file=sys.stderr, flush=True)
    if a.tune_save and ctx.rank == 0:
        from pytorch_imageclassification_distributed_amd.ops import hip
        print(f"[bench] saved {hip.save_tuning(a.tune_save)} kernel choices to {a.tune_save}", file=sys.stderr)
    extra = {}
    if ctx.device.type == "cuda":
        # allocator steady state: every device malloc / free in the timed steps is a device sync
        extra["timed_device_malloc"] = m1["device_malloc"] - m0["device_malloc"]
        extra["timed_device_free"] = m1["device_free"] - m0["device_free"]
    if comm_t is not None:
        from pytorch_imageclassification_distributed_amd.parallel import comm_timer
        comm_timer.uninstall()
        extra.update(comm_t.summary())  # rank-local means; reported for the slowest rank below
        if tr.reducer is not None:
            extra["bucket_mb"] = [round(v, 2) for v in tr.reducer.bucket_sizes_mb()]
    if sync_bn and ctx.world_size > 1:
        extra.update(_syncbn_checks(tr, ctx))
    t = torch.tensor([dt], dtype=torch.float64, device=ctx.device)
    if ctx.world_size > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        extra = _from_slowest_rank(extra, dt, ctx, a.steps)
    dt = float(t.item())
    loss_val = float(last.item())
    if ctx.rank == 0:
        imgs = a.batch * ctx.world_size * a.steps
        value = imgs / dt
        base = (load_baseline(ctx.world_size, a.batch, a.model, a.image_size)
                if a.dtype == "bf16" and a.device == "cuda" else None)
        metric = METRIC if (a.model, a.image_size, a.dtype, a.device) == ("resnet50", 224, "bf16", "cuda") else \
            f"images/sec (whole node) {a.model} {a.image_size}x{a.image_size} {a.dtype} MI355X"
        if a.device == "cpu":
            metric = "CPU REHEARSAL of the multi-rank path (gloo, fp32, not a benchmark): " + metric
        if os.environ.get("IMGCLS_DIAG_SKIP_WGRAD", "0") == "1":  # a diagnostic, never a benchmark number
            metric, base = "DIAGNOSTIC (weight gradients skipped, invalid as a benchmark): " + metric, None
        if os.environ.get("IMGCLS_DIAG_SKIP_GRAD_COMM", "0") == "1" and ctx.world_size > 1:
            metric, base = "DIAGNOSTIC (gradient all-reduce skipped, invalid as a benchmark): " + metric, None
        print(json.dumps({
            "metric": metric, "value": round(value, 2), "unit": "images/sec",
            "n_gpus": ctx.world_size, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": round(value / base, 4) if base else None,
            "dtype": (("fp8 (MX-FP8 e4m3 forward convolutions, bf16 backward and BN)" if a.dtype == "fp8" else a.dtype)
                      if a.device == "cuda" else "fp32 (cpu rehearsal, not a benchmark)"),
            "data": ("synthetic (on-device random images, random-init weights)" if a.data == "device" else
                     "synthetic (pinned uint8 host batches, H2D copy + normalisation in the timed loop, "
                     "random-init weights)"),
            "config": {"model": a.model, "global_batch": a.batch * ctx.world_size,
                       "per_gpu_batch": a.batch, "seq_len": None, "image_size": a.image_size,
                       "num_classes": a.num_classes, "parallelism": f"dp{ctx.world_size}",
                       "sync_bn": sync_bn, "syncbn_comm": ("peer" if tr.syncbn_peer else "rccl") if sync_bn else None,
                       "compute": a.compute, "optimizer": "adam", "hip_graph": use_graph,
                       "grad_comm": (getattr(tr, "comm_backend", a.comm_backend) if ctx.world_size > 1 else None),
                       "final_loss": round(loss_val, 5)},
            **extra,
        }), flush=True)
    destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
