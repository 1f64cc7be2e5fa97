"""CLI / config for ``train.py``.

The reference has exactly three flags (train.py:27-31): ``--local_rank`` (int,
default 0), ``--datadir`` (required), ``--batchsize`` (int, default 4).  They are
kept with the same names and defaults (``--local-rank`` is accepted too, A7).
Everything the reference hard-codes becomes a flag whose default equals the
reference constant: model ``inceptionv3`` (train.py:122), image
size 299 (:110), lr 5e-6 (:127), milestones 50/80 and gamma 0.5 (:156), class
weights 3,3,10,1,4,4,5 (:157), 100 epochs (:161), 6 workers (:114), val batch 1
(:118), aux weight 0.4 (:52), ``dtmodel/cp`` (:136), latest every 5 epochs (:183).
"""
from __future__ import annotations

import argparse

REF_CLASS_WEIGHTS = (3.0, 3.0, 10.0, 1.0, 4.0, 4.0, 5.0)
GRAPH_AUTO_MAX_BATCH = 64  # --hip-graph auto: largest per-GPU batch that replays the step as a graph


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X-native distributed image classification trainer")
    # --- reference flags (train.py:27-31)
    p.add_argument("--local_rank", "--local-rank", dest="local_rank", default=0, type=int)
    p.add_argument("--datadir", default="", help="ImageFolder root with train/ and valid/ (required unless --synthetic)")
    p.add_argument("--batchsize", default=4, type=int, help="per-process batch size")
    # --- reference constants as flags
    p.add_argument("--model", default="inceptionv3")
    p.add_argument("--image-size", type=int, default=None, help="default: 299 for inceptionv3, 224 resnets, native for efficientnet")
    p.add_argument("--lr", type=float, default=0.5e-5)
    p.add_argument("--epochs", type=int, default=100)
    p.add_argument("--milestones", type=int, nargs="*", default=[50, 80])
    p.add_argument("--gamma", type=float, default=0.5)
    p.add_argument("--class-weights", default="auto",
                   help="comma list, 'auto' (reference weights if 7 classes else uniform) or 'none'")
    p.add_argument("--num-workers", type=int, default=6)
    p.add_argument("--loader", default="auto", choices=["auto", "native", "python"],
                   help="image-folder loading: native C++ threads (PNG), the Python DataLoader, or auto")
    p.add_argument("--val-batchsize", type=int, default=1)
    p.add_argument("--aux-weight", type=float, default=0.4)
    p.add_argument("--ckpt-dir", default="dtmodel/cp")
    p.add_argument("--latest-every", type=int, default=5)
    # --- new
    p.add_argument("--synthetic", action="store_true", help="synthetic data instead of --datadir")
    p.add_argument("--synthetic-train-size", type=int, default=512)
    p.add_argument("--synthetic-val-size", type=int, default=128)
    p.add_argument("--num-classes", type=int, default=None, help="default: from dataset (synthetic: 7)")
    p.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    p.add_argument("--backend", default="auto", help="process group backend: auto|rccl|nccl|gloo")
    p.add_argument("--compute", default="auto", choices=["auto", "hip", "torch"],
                   help="hip = native kernels (GPU default); torch = ATen reference stack")
    p.add_argument("--dtype", default="bf16", choices=["bf16", "fp32", "fp8"],
                   help="GPU compute dtype: bf16 (fp32 master weights); fp8 = experimental MX-FP8 forward "
                        "convolutions (e4m3 + E8M0 per 32 channels) where Cin %% 128 == 0, bf16 elsewhere and in "
                        "backward (no measurable speed-up: README); fp32 = the ATen path only (--compute torch)")
    p.add_argument("--sync-bn", dest="sync_bn", action="store_true", default=True)
    p.add_argument("--no-sync-bn", dest="sync_bn", action="store_false")
    p.add_argument("--syncbn-comm", default="auto", choices=["auto", "peer", "rccl"],
                   help="SyncBN statistics transport: one-shot peer all-reduce over xGMI IPC buffers (peer), "
                        "torch.distributed / RCCL (rccl), or peer when all ranks share a host and it self-checks (auto)")
    p.add_argument("--syncbn-check-every", type=int, default=100,
                   help="every N train steps (and at each epoch end) check that all ranks hold bitwise-equal BN "
                        "running statistics and that no SyncBN peer exchange timed out (0: epoch end only)")
    p.add_argument("--bucket-mb", type=float, default=32.0)
    p.add_argument("--tail-bucket-mb", type=float, default=4.0,
                   help="cut the last gradient bucket (the last gradients of backward: stem + first stage) into "
                        "pieces of at most this many MiB, so only the final piece's all-reduce sits after backward "
                        "(0: one bucket)")
    p.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"])
    p.add_argument("--comm-backend", default="pg", choices=["pg", "rccl"],
                   help="gradient buckets: torch.distributed's ProcessGroupNCCL (pg) or our C++ RCCL communicator "
                        "(rccl: one comm stream behind the weight-gradient stream, parallel/rccl.py; a host "
                        "watchdog ends the run if its collectives stall past --timeout-min).  rccl needs SyncBN "
                        "off or on the peer transport: with SyncBN on RCCL the run falls back to pg (two "
                        "communicators' collectives in flight on the same GPUs have no progress guarantee)")
    p.add_argument("--steps-per-epoch", type=int, default=None, help="cap on train steps per epoch")
    p.add_argument("--val-steps", type=int, default=None, help="cap on validation steps")
    p.add_argument("--resume", default="best",
                   help="best (reference behaviour) | latest | auto | none | <path>")
    p.add_argument("--log-interval", type=int, default=1,
                   help="host-side loss readback every N steps (1 = reference per-step semantics)")
    p.add_argument("--no-progress", action="store_true", help="disable tqdm progress bar")
    p.add_argument("--metrics-file", default=None, help="rank-0 JSONL metrics output")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--exact-val", action="store_true", help="mask DistributedSampler padding in validation (A15)")
    p.add_argument("--pretrained", default=None, help="local torchvision-layout state_dict to initialise the backbone")
    p.add_argument("--step-timers", action="store_true",
                   help="per-phase step timing (data/forward/backward/comm/optimizer) into --metrics-file")
    p.add_argument("--profile-steps", type=int, default=0, help="torch.profiler trace over this many train steps")
    p.add_argument("--profile-start", type=int, default=5, help="first profiled global step")
    p.add_argument("--profile-dir", default="profiles/trace", help="where trace_rank<r>.json is written")
    p.add_argument("--broadcast-buffers", action="store_true",
                   help="DDP broadcast_buffers parity (X3): broadcast BN buffers from rank 0 before each forward")
    p.add_argument("--deterministic", action="store_true",
                   help="bitwise-reproducible GPU kernels (no split-K / cross-block fp32 atomics; slower)")
    p.add_argument("--timeout-min", type=float, default=10.0, help="process-group timeout (minutes)")
    p.add_argument("--hip-graph", nargs="?", const="on", default="auto", choices=["on", "off", "auto"],
                   help="capture the whole training step once and replay it as one HIP graph (host-bound steps; "
                        "at N > 1 forward + backward with the SyncBN peer exchanges, then one flat gradient "
                        "all-reduce and Adam); a batch of another shape runs eagerly.  auto = on at per-GPU "
                        f"batch <= {GRAPH_AUTO_MAX_BATCH} (Inception-v3 @299: b4 466 vs 164 img/s eager, b32 "
                        "2943 vs 1978; at b128 eager wins, profiles/history/r6_bench_host_data_and_inception_small_batch.jsonl)")
    return p


def hip_graph_enabled(args, world_size: int) -> bool:
    """Whether ``--hip-graph`` (on / off / auto) replays the training step as a HIP graph."""
    mode = getattr(args, "hip_graph", "off")
    if mode is True:
        mode = "on"
    if mode in (False, None, "off"):
        return False
    return mode == "on" or args.batchsize <= GRAPH_AUTO_MAX_BATCH


def parse_class_weights(spec: str, num_classes: int):
    if spec == "none":
        return None
    if spec == "auto":
        return list(REF_CLASS_WEIGHTS) if num_classes == len(REF_CLASS_WEIGHTS) else None
    w = [float(x) for x in spec.split(",")]
    if len(w) != num_classes:
        raise ValueError(f"--class-weights has {len(w)} entries, dataset has {num_classes} classes")
    return w
