"""Training engine with the reference's semantics (reference train.py:36-188).

Per training step (reference train.py:44-73):
  H2D copy -> forward (Inception: ``CE(logits) + 0.4*CE(aux)``) -> loss
  all-reduce SUM / world -> meter update -> rank-0 progress text
  ``Epoch: {e}; Loss {val:.4f}|({avg:.4f})`` -> zero_grad -> backward -> step.
Per epoch (train.py:161-188): ``sampler.set_epoch`` -> train -> scheduler.step
-> validate (top-1 %, all ranks combined) -> rank 0 saves ``best_model`` on
improvement and ``latest_model`` every 5 epochs.

Execution paths:
* ``compute='hip'`` (GPU default): our kernels, our bucketed RCCL reducer
  (``parallel.GradReducer``), our SyncBN, fused Adam.
* ``compute='torch'`` on GPU: the *reference stack* - torch DDP +
  nn.SyncBatchNorm + bf16 autocast over ATen/MIOpen - used to measure the
  baseline on the same box.
* CPU: ATen reference ops, gloo, our reducer/SyncBN (torch SyncBN is GPU-only).

Host syncs: the loss readback happens every ``log_interval`` steps (1 =
reference behaviour, A21); validation accumulates correct/total on device and
all-reduces two integers (A14) instead of per-sample ``.cpu()`` + pickle.
"""
from __future__ import annotations

import collections
import math
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn as nn
from torch.utils.data import DataLoader
from torch.utils.data.distributed import DistributedSampler

from ..data import CudaPrefetcher, ImageDataset, NativeFolderLoader, SyntheticImageDataset, use_native
from ..models import DEFAULT_IMAGE_SIZE, Classifier
from ..ops import functional as Fx
from ..ops.grad_arena import GradArena
from ..parallel import (GradReducer, check_peer_errors, check_syncbn_consistency, comm_timer, convert_sync_batchnorm,
                        setup_peer_syncbn)
from ..utils import (BEST, LATEST, AccuracyCounter, DeviceMeter, JsonlLogger, load_checkpoint,
                     load_model_state, resolve_resume, save_checkpoint)
from ..utils.checkpoint import gather_rng_states, restore_rank_rng
from ..utils.timers import PhaseTimer
from .config import hip_graph_enabled, parse_class_weights
from .optim import FusedAdam, MultiStepLR

# training steps the host may have enqueued ahead of the GPU (Trainer._throttle; 0 = unbounded).  Unset: 2, or
# 3 when a step's peak allocation is under SMALL_STEP_FRACTION of the device (host-bound small-memory steps; round
# 4 measured Inception-v3 b256 8323 -> 8400 img/s with 4, profiles/history/r7d_*).  Round 6 re-measured 2 / 3 / 4 on
# the current build: throughput equal within noise, but with 4 the caching allocator kept mapping blocks in the
# timed region (ResNet-101 b256: 118 hipMallocs in 20 steps, EfficientNet-B0 b256: 23) while 3 left 0 there
# (profiles/r15x_inflight_alloc_ab.txt).  ResNet-50 b1024 at 44 GiB keeps 2.
MAX_INFLIGHT_STEPS = int(os.environ.get("IMGCLS_MAX_INFLIGHT_STEPS", "-1"))
SMALL_STEP_FRACTION = 0.1


def _is_inception(name: str) -> bool:
    return "inception" in name


class Trainer:
    def __init__(self, args, ctx):
        self.args, self.ctx = args, ctx
        self.dev = ctx.device
        torch.manual_seed(args.seed)
        if args.compute != "auto":
            Fx.set_backend(args.compute)
        self.hip = self.dev.type == "cuda" and Fx.get_backend() != "torch"
        if self.hip and getattr(args, "dtype", "bf16") == "fp32":
            # the native kernels store activations / weight shadows in bf16 (fp32 accumulation, fp32 master
            # weights, fp32 BN statistics and head); an fp32 request must not silently run bf16
            raise SystemExit("--dtype fp32: the HIP kernels compute in bf16 with fp32 accumulation; for the "
                             "reference's fp32 numerics use --compute torch --dtype fp32 (ATen fp32, no autocast)")
        if self.hip:
            from ..ops import hip as _hipmod
            _hipmod.set_fp8(getattr(args, "dtype", "bf16") == "fp8")
        if getattr(args, "deterministic", False):
            torch.backends.cudnn.deterministic = True
            torch.backends.cudnn.benchmark = False
            if self.hip:
                from ..ops import hip as _hip
                _hip.set_deterministic(True)
        self.name = args.model
        self.image_size = args.image_size or DEFAULT_IMAGE_SIZE.get(args.model, 224)
        self._build_data()
        self._build_model()
        self.input_fn = None
        spec = getattr(self.model.encoder, "input_spec", None) if hasattr(self.model, "encoder") else None
        if self.hip and spec is not None:
            # loaders that deliver uint8 batches convert them to the model's input in one kernel on their copy
            # stream (normalisation, layout / space-to-depth, transform_input)
            import functools
            from ..data.folder import IMAGENET_MEAN, IMAGENET_STD
            from ..ops import hip as _hipops
            self.input_fn = functools.partial(_hipops.input_from_u8, spec=spec(), mean=IMAGENET_MEAN,
                                              std=IMAGENET_STD)
            for ld in (getattr(self, "train_loader", None), getattr(self, "val_loader", None)):
                if ld is not None and hasattr(ld, "input_fn"):
                    ld.input_fn = self.input_fn
        if ctx.world_size > 1:
            # the weights are rank 0's (broadcast at construction); from here each rank draws its own dropout /
            # drop-connect masks, as unseeded DDP ranks do (a checkpoint keeps every rank's streams: rng_ranks)
            torch.manual_seed(args.seed + 1_000_003 * ctx.rank)

    # ------------------------------------------------------------------ data
    def _build_data(self):
        a = self.args
        if a.synthetic:
            nc = a.num_classes or 7
            self.train_ds = SyntheticImageDataset(a.synthetic_train_size, nc, self.image_size, seed=a.seed)
            self.val_ds = SyntheticImageDataset(a.synthetic_val_size, nc, self.image_size, seed=a.seed + 1)
        else:
            if not a.datadir:
                raise SystemExit("--datadir is required unless --synthetic is given")
            self.train_ds = ImageDataset(a.datadir, "train", self.image_size)
            self.val_ds = ImageDataset(a.datadir, "valid", self.image_size)
        self.num_classes = a.num_classes or (self.train_ds.num_classes if not a.synthetic else 7)
        pin = self.dev.type == "cuda"
        self.train_sampler = DistributedSampler(self.train_ds, num_replicas=self.ctx.world_size,
                                                rank=self.ctx.rank, seed=a.seed)
        self.val_sampler = DistributedSampler(self.val_ds, num_replicas=self.ctx.world_size,
                                              rank=self.ctx.rank, seed=a.seed)
        mode = getattr(a, "loader", "auto")
        if mode == "native" and not (use_native(self.train_ds) and use_native(self.val_ds)):
            raise SystemExit("--loader native needs PNG image folders and the built extension")
        if mode == "native" or (mode == "auto" and use_native(self.train_ds) and use_native(self.val_ds)):
            # C++ decode/augment threads -> pinned uint8 ring -> GPU normalisation (data/native.py)
            workers = max(a.num_workers, 1)
            self.train_loader = NativeFolderLoader(self.train_ds, self.train_sampler, a.batchsize, self.dev,
                                                   workers=workers, seed=a.seed)
            self.val_loader = NativeFolderLoader(self.val_ds, self.val_sampler, a.val_batchsize, self.dev,
                                                 workers=workers, seed=a.seed)
            return
        self.train_loader = DataLoader(self.train_ds, batch_size=a.batchsize, shuffle=False,
                                       num_workers=a.num_workers, pin_memory=pin,
                                       sampler=self.train_sampler, drop_last=False,
                                       persistent_workers=a.num_workers > 0)
        self.val_loader = DataLoader(self.val_ds, batch_size=a.val_batchsize, shuffle=False,
                                     num_workers=a.num_workers, pin_memory=pin, sampler=self.val_sampler)

    # ------------------------------------------------------------------ model
    def _build_model(self):
        a, ctx = self.args, self.ctx
        model = Classifier(self.name, self.num_classes, pretrained=a.pretrained).to(self.dev)
        self.ddp = None
        self.syncbn_peer = False
        self.reducer = None
        self.arena = None
        self.autocast = False
        if self.dev.type == "cuda" and not self.hip:
            # reference stack: torch DDP + SyncBatchNorm (+ bf16 autocast).  bf16: channels-last (MIOpen's fast
            # layout); fp32 keeps the reference's own NCHW layout - MIOpen's fp32 channels-last backward faulted
            # the GPU on EfficientNet-B0 (illegal memory access, gpurun_out/r5e_pytest_learning.log)
            if a.dtype != "fp32":
                model = model.to(memory_format=torch.channels_last)
            if a.sync_bn and ctx.world_size > 1:
                model = nn.SyncBatchNorm.convert_sync_batchnorm(model)
            self.autocast = a.dtype == "bf16"
            net = model
            if ctx.world_size > 1:
                net = nn.parallel.DistributedDataParallel(model, device_ids=[ctx.local_rank],
                                                          output_device=ctx.local_rank,
                                                          bucket_cap_mb=a.bucket_mb,
                                                          broadcast_buffers=getattr(a, "broadcast_buffers", False))
            self.net = net
        else:
            if self.hip:
                model = model.to(memory_format=torch.channels_last)
            if a.sync_bn:
                # a communicator of its own: the 2x53 latency-bound SyncBN collectives must not queue
                # behind the reducer's 32 MiB gradient buckets on the default group's RCCL stream
                grp = dist.new_group(list(range(ctx.world_size))) if ctx.world_size > 1 else None
                convert_sync_batchnorm(model, grp)
                # one-shot xGMI peer all-reduce for the 2x53 statistics exchanges (parallel/peer.py)
                self.syncbn_peer = self.hip and grp is not None and setup_peer_syncbn(
                    grp, self.dev, getattr(a, "syncbn_comm", "auto"))
            if ctx.world_size > 1:
                comm = torch.bfloat16 if a.comm_dtype == "bf16" else None
                backend = getattr(a, "comm_backend", "pg") if self.dev.type == "cuda" else "pg"
                if backend == "rccl" and a.sync_bn and not self.syncbn_peer:
                    # SyncBN's statistics would go through ProcessGroupNCCL while the buckets ride our own
                    # communicator: two communicators' collectives in flight on the same GPUs, in no common
                    # order, have no progress guarantee - keep every collective on the process group
                    if ctx.is_main:
                        print("[imgcls] --comm-backend rccl needs SyncBN off or on the peer transport; "
                              "gradient buckets use the process group (pg)", file=sys.stderr, flush=True)
                    backend = "pg"
                self.comm_backend = backend
                self.reducer = GradReducer(model, bucket_cap_mb=a.bucket_mb, comm_dtype=comm, comm=backend,
                                           timeout_s=60.0 * getattr(a, "timeout_min", 10.0),
                                           tail_bucket_mb=getattr(a, "tail_bucket_mb", 4.0))
                self.arena = self.reducer.arena
            elif self.hip:
                params = [p for p in model.parameters() if p.requires_grad]
                self.arena = GradArena(params, list(reversed(range(len(params)))))
            self.net = model
        self.model = model
        self.optimizer = FusedAdam(model.parameters(), lr=a.lr)
        self.scheduler = MultiStepLR(self.optimizer, milestones=a.milestones, gamma=a.gamma)
        w = parse_class_weights(a.class_weights, self.num_classes)
        self.class_weight = torch.tensor(w, dtype=torch.float32, device=self.dev) if w else None
        self.best_score = 0.0
        self.start_epoch = 0
        self.global_step = 0
        self.timer = PhaseTimer(getattr(a, "step_timers", False), self.dev)
        self.step_stream = None
        if self.hip and os.environ.get("IMGCLS_HIPRIO_STEP", "1") == "1":
            lo, hi = torch.cuda.Stream.priority_range()
            if hi < lo:  # the device has a priority above the default
                self.step_stream = torch.cuda.Stream(device=self.dev, priority=hi)
        self.log = JsonlLogger(getattr(a, "metrics_file", None), self.ctx.is_main)
        self._prof = None
        self._graph = None  # captured whole-step HIP graph (``capture_step``)
        self._g_coll = False  # the captured step carries the gradient collectives (native RCCL communicator)
        self._eager_steps = 0  # eager training steps run by this process (graph capture waits for 2)
        self._steps_enqueued = 0
        self._auto_inflight = None  # MAX_INFLIGHT_STEPS unset: chosen from the steady-state peak allocation
        self._inflight = collections.deque()  # end-of-step events of the steps the GPU has not finished

    # ------------------------------------------------------------------ step
    def compute_loss(self, images, labels):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.autocast):
            out = self.net(images)
        if _is_inception(self.name) and isinstance(out, tuple):
            return (Fx.cross_entropy(out[0], labels, self.class_weight)
                    + self.args.aux_weight * Fx.cross_entropy(out[1], labels, self.class_weight))
        return Fx.cross_entropy(out, labels, self.class_weight)

    def train_step(self, images, labels):
        """forward + loss + backward + (overlapped) all-reduce + Adam.  Returns the local loss.

        Phases are bracketed for ``--step-timers`` (device events) and named for ``--profile-steps``
        (torch.profiler ranges: imgcls::forward / backward / comm_wait / optimizer).

        On the HIP path the step runs on a high-priority HIP stream: the weight gradients go to a
        normal-priority side stream (ops/hip.py, "weight gradients on a side stream"), so the
        dispatcher hands free CUs to the critical dgrad -> BN-backward chain first and the weight
        GEMMs fill the rest (ResNet-50 b512: +1.5 % over one stream; the side stream at equal priority
        was 1.8 % slower than one stream)."""
        self._throttle()
        st = self.step_stream
        if st is None:
            loss = self._train_step(images, labels)
            self._step_enqueued()
            return loss
        caller = torch.cuda.current_stream(self.dev)
        st.wait_stream(caller)
        with torch.cuda.stream(st):
            loss = self._train_step(images, labels)
        caller.wait_stream(st)
        loss.record_stream(caller)
        self._step_enqueued()
        return loss

    def _throttle(self) -> None:
        """Keep at most MAX_INFLIGHT_STEPS steps enqueued ahead of the GPU (a host wait on the oldest step's
        end event).  The host enqueues a ResNet-50 b1024 step in ~10 ms and the GPU runs it in ~75 ms, so an
        unthrottled host runs many steps ahead.  Every tensor handed to the weight-gradient side stream
        (``record_stream``) then stays unusable until the GPU reaches its event, so the caching allocator
        keeps mapping new blocks for the steps in flight.  Round 3 measured ResNet-50 b1024 at 44 GiB
        allocated but 286 GiB reserved; at the 288 GB limit the allocator frees its whole cache with
        device syncs and re-maps each block: 1.6 s steps, the b1536 / b2048 slowdown of round 2
        (docs/DESIGN.md).  Two steps in flight keep the GPU fed and bound the cache."""
        limit = self._inflight_limit()
        if limit <= 0:
            return
        while len(self._inflight) >= limit:
            self._inflight.popleft().synchronize()

    def _inflight_limit(self) -> int:
        if self.dev.type != "cuda" or MAX_INFLIGHT_STEPS == 0:
            return 0
        if MAX_INFLIGHT_STEPS > 0:
            return MAX_INFLIGHT_STEPS
        if self._auto_inflight is None:
            if self._steps_enqueued < 2:  # the first steps tune kernels: their peak is not the steady one
                return 2
            if self._steps_enqueued == 2:  # drop the tuning steps' peak; decide from the next step's
                torch.cuda.reset_peak_memory_stats(self.dev)
                return 2
            total = torch.cuda.get_device_properties(self.dev).total_memory
            small = torch.cuda.max_memory_allocated(self.dev) < SMALL_STEP_FRACTION * total
            self._auto_inflight = 3 if small else 2
        return self._auto_inflight

    def _step_enqueued(self) -> None:
        self._steps_enqueued += 1
        if self._inflight_limit() > 0:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.dev))
            self._inflight.append(ev)

    # ------------------------------------------------------------------ HIP graph
    def capture_step(self, images, labels) -> None:
        """Capture one whole training step (forward, loss, backward, fused Adam) into a HIP graph that
        ``graph_step`` replays: one launch per step instead of ~1000 host-side op dispatches (Inception-v3
        and EfficientNet steps are host-bound in eager mode).  Call after enough eager steps that every
        kernel shape is tuned (the tuner never runs under capture).  Single process (world 1): the
        graph carries no collectives.  Inputs are copied into static buffers on every replay; the
        learning rate is a kernel argument of the captured Adam launch, so a scheduler change
        re-captures (``graph_step`` checks).

        At N > 1 the graph holds forward + loss + backward, SyncBN exchanges included: the one-shot peer
        kernels take their call numbers from a device counter (``csrc/peer.hip``), so every replay
        exchanges fresh statistics.  With the native RCCL communicator (``--comm-backend rccl``) the bucket
        collectives are captured as well: the hooks run once, at capture, and enqueue each bucket's all-reduce
        on the comm stream, which forks from the capture stream at that point and joins back before the
        captured Adam, so on replay the collectives overlap the rest of backward exactly as in an eager step.
        ProcessGroupNCCL's collectives cannot sit in a graph, so on that backend the capture defers them (the
        hooks only fill the arena) and after each replay one flat all-reduce of the gradient arena and the
        fused Adam run eagerly (``graph_step``): ~1000 host dispatches become a replay plus three."""
        if not self.graph_capable():
            raise RuntimeError("capture_step: needs the HIP path and, at N > 1, SyncBN off or on the peer "
                               "transport (no process-group collective inside the step) and no buffer broadcast")
        self._g_x = images.detach().clone()
        for attr in ("_imgcls_s2d", "_imgcls_prepared"):  # loader-converted input (input_from_u8) stays marked
            if hasattr(images, attr):
                setattr(self._g_x, attr, getattr(images, attr))
        self._g_y = labels.detach().clone()
        self._g_lrs = tuple(g["lr"] for g in self.optimizer.param_groups)
        st = self.step_stream if self.step_stream is not None else torch.cuda.Stream(device=self.dev)
        # in-graph collectives (native RCCL communicator): the bucket all-reduces are captured on the comm
        # stream's fork and overlap the rest of the captured backward; Adam is captured too
        self._g_coll = self.reducer is not None and self.reducer.graph_collectives
        split = self.ctx.world_size > 1 and not self._g_coll
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        if split:
            self.reducer.deferred = True
        with torch.cuda.graph(g, stream=st):
            self._g_loss = self._train_step(self._g_x, self._g_y, update=not split)
        if split:  # replays run no hooks; an eager step in between (another batch shape) reduces as usual
            self.reducer.deferred = False
        if self.reducer is not None:
            self.reducer.reset_after_capture()
        torch.cuda.synchronize(self.dev)
        self._graph, self._g_stream, self._g_split = g, st, split

    def graph_capable(self) -> bool:
        """Whole-step replay works: HIP path, and at N > 1 nothing inside the step that talks to the
        process group (SyncBN over the peer kernels or off, no per-step buffer broadcast)."""
        if not self.hip:
            return False
        if self.ctx.world_size == 1:
            return True
        return (self.reducer is not None and not getattr(self.args, "broadcast_buffers", False)
                and (not self.args.sync_bn or self.syncbn_peer))

    def graph_step(self, images, labels):
        """Replay the captured step on new inputs (same shapes); returns the step's loss tensor, valid
        until the next replay is enqueued."""
        # the learning rate is baked into a captured Adam launch; at N > 1 with deferred collectives Adam runs
        # eagerly after the replay and reads the current lr, so a schedule change needs no re-capture there
        if self._graph is None or (not self._g_split and
                                   tuple(g["lr"] for g in self.optimizer.param_groups) != self._g_lrs):
            self._graph = None
            self.capture_step(images, labels)
        self._throttle()
        st = self._g_stream
        caller = torch.cuda.current_stream(self.dev)
        st.wait_stream(caller)
        with torch.cuda.stream(st):
            self._g_x.copy_(images, non_blocking=True)
            self._g_y.copy_(labels, non_blocking=True)
            self._graph.replay()
            if self._g_split:  # N > 1: the gradients of the replayed backward, summed once, then Adam
                self.optimizer.step(grad_scale=self.reducer.flat_all_reduce())
            elif self._g_coll:  # the replay carried the collectives: give them a deadline
                self.reducer.arm_watchdog(st)
        caller.wait_stream(st)
        images.record_stream(st)
        labels.record_stream(st)
        self._step_enqueued()
        return self._g_loss

    def _epoch_step(self, images, labels, index: int):
        """``--hip-graph``: eager for the first two steps this process runs (every kernel shape gets tuned;
        counted per process, so a resumed run warms up too), then capture once - on a full batch of the
        loader's batch size, never on an epoch's short last batch - and replay; a batch of another shape
        runs eagerly."""
        use = hip_graph_enabled(self.args, self.ctx.world_size) and self.graph_capable() and not self._prof
        if use:
            if self._graph is not None:
                if self._g_x.shape == images.shape and self._g_y.shape == labels.shape:
                    return self.graph_step(images, labels)
            elif self._eager_steps >= 2 and images.shape[0] == self.args.batchsize:
                return self.graph_step(images, labels)
        self._eager_steps += 1
        return self.train_step(images, labels)

    def _train_step(self, images, labels, update: bool = True):
        """One step; ``update=False`` stops after backward (the N > 1 graph capture: the gradient reduce and
        Adam run after each replay)."""
        rf = torch.profiler.record_function
        timer = self.timer
        ct = comm_timer._TIMER if (self.dev.type == "cuda" and not torch.cuda.is_current_stream_capturing()) else None
        if ct is not None:
            ct.begin()
        if self.reducer is not None and getattr(self.args, "broadcast_buffers", False):
            self.reducer.sync_buffers()
        with rf("imgcls::forward"):
            loss = self.compute_loss(images, labels)
        timer.mark("forward")
        with rf("imgcls::backward"):
            self.optimizer.zero_grad(set_to_none=True)
            if self.arena is not None:
                self.arena.begin()  # one memset; backward kernels write into persistent slots
            loss.backward()
            if self.hip:
                from ..ops import hip as _hip
                _hip.join_side_streams()  # (normally already done by the engine callback)
        timer.mark("backward")
        if not update:
            return loss.detach()
        with rf("imgcls::comm_wait"):
            scale = self.reducer.finish() if self.reducer is not None else 1.0
        timer.mark("comm_wait")
        with rf("imgcls::optimizer"):
            self.optimizer.step(grad_scale=scale)
        timer.mark("optimizer")
        if ct is not None:
            ct.end()
        return loss.detach()

    def reduce_loss(self, loss):
        """Reference train.py:59-63: all-reduce SUM / world (enqueued, no host sync)."""
        red = loss.clone().float()
        if self.ctx.world_size > 1:
            dist.all_reduce(red, op=dist.ReduceOp.SUM)
            red /= self.ctx.world_size
        return red

    def _profile_tick(self):
        """Start / stop the torch.profiler window [profile_start, profile_start + profile_steps)."""
        a = self.args
        n = getattr(a, "profile_steps", 0)
        if n <= 0:
            return
        if self.global_step == a.profile_start and self._prof is None:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if self.dev.type == "cuda":
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts)
            self._prof.__enter__()
        elif self.global_step == a.profile_start + n and self._prof is not None:
            if self.dev.type == "cuda":
                torch.cuda.synchronize()
            self._prof.__exit__(None, None, None)
            os.makedirs(a.profile_dir, exist_ok=True)
            path = os.path.join(a.profile_dir, f"trace_rank{self.ctx.rank}.json")
            self._prof.export_chrome_trace(path)
            if self.ctx.is_main:
                print(f"profiler trace written to {path}", flush=True)
            self._prof = False  # one window per run

    # ------------------------------------------------------------------ epochs
    def _loader(self, loader):
        if isinstance(loader, NativeFolderLoader):  # copies + normalises on its own stream
            return loader
        return CudaPrefetcher(loader, self.dev) if self.dev.type == "cuda" else loader

    def train_epoch(self, epoch: int):
        a = self.args
        self.net.train()
        meter = DeviceMeter(self.dev)
        show = self.ctx.is_main and not a.no_progress
        it = self._loader(self.train_loader)
        bar = None
        if show:
            from tqdm import tqdm
            bar = tqdm(total=len(self.train_loader) if a.steps_per_epoch is None
                       else min(len(self.train_loader), a.steps_per_epoch), file=sys.stdout)
        t_log, n_log = time.perf_counter(), 0
        self.timer.mark("data")
        for index, data in enumerate(it):
            if a.steps_per_epoch is not None and index >= a.steps_per_epoch:
                break
            images, labels = data["image"], data["label"]
            if images.device != self.dev:
                images = images.to(self.dev, non_blocking=True)
                labels = labels.to(self.dev, non_blocking=True)
            self.timer.mark("data")
            self._profile_tick()
            loss = self._epoch_step(images, labels, index)
            meter.update(self.reduce_loss(loss), images.size(0))
            self.global_step += 1
            n_log += images.size(0)
            every = getattr(a, "syncbn_check_every", 100)
            if self.syncbn_peer and every > 0 and self.global_step % every == 0:
                # a timed-out SyncBN peer exchange is fatal; ranks must agree bitwise (parallel/peer.py) -
                # its own interval: the guard is a collective plus a host sync, not a per-step cost
                check_peer_errors(f"epoch {epoch} step {index}")
                check_syncbn_consistency(self.model, None, f"epoch {epoch} step {index}")
            if (index + 1) % max(a.log_interval, 1) == 0:
                if self.reducer is not None:
                    self.reducer.check()  # native communicator async error (no-op on the process group)
                if bar is not None:
                    bar.set_description(f"Epoch: {epoch}; Loss {meter.val:.4f}|({meter.avg:.4f})")
                if self.timer.enabled:
                    tot = self.timer.flush()
                    now = time.perf_counter()
                    steps = max(a.log_interval, 1)
                    self.log.log(kind="step", epoch=epoch, step=self.global_step,
                                 images_per_sec=n_log * self.ctx.world_size / max(now - t_log, 1e-9),
                                 **{f"ms_{k}": v / steps for k, v in tot.items()})
                    self.timer.reset()
                    t_log, n_log = now, 0
            if bar is not None:
                bar.update(1)
        if bar is not None:
            bar.set_description(f"Epoch: {epoch}; Loss {meter.val:.4f}|({meter.avg:.4f})")
            bar.close()
        if self.syncbn_peer:
            check_peer_errors(f"end of epoch {epoch}")
            check_syncbn_consistency(self.model, None, f"end of epoch {epoch}")
        return meter.avg if meter.count else float("nan")

    @torch.no_grad()
    def val_epoch(self, epoch: int) -> float:
        a = self.args
        self.net.eval()
        acc = AccuracyCounter(self.dev)
        n_real = len(self.val_ds)
        rank, world = self.ctx.rank, self.ctx.world_size
        for index, data in enumerate(self._loader(self.val_loader)):
            if a.val_steps is not None and index >= a.val_steps:
                break
            images, labels = data["image"], data["label"]
            if images.device != self.dev:
                images = images.to(self.dev, non_blocking=True)
                labels = labels.to(self.dev, non_blocking=True)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.autocast):
                out = self.net(images)
            valid = None
            if a.exact_val:
                # sampler index i*world+rank >= len(dataset) is DistributedSampler padding
                pos = index * a.val_batchsize + torch.arange(labels.numel(), device=self.dev)
                valid = (pos * world + rank) < n_real
            acc.update(out.float(), labels, valid)
        counts = torch.stack([acc.correct, acc.total]).to(torch.float64)
        if world > 1:
            dist.all_reduce(counts)
        comb = float(counts[0] / counts[1].clamp(min=1) * 100.0)
        if self.ctx.is_main:
            print(f"Validation Accuracy {comb}", flush=True)
        return comb

    # ------------------------------------------------------------------ ckpt
    def ckpt_path(self, which: str) -> str:
        return os.path.join(self.args.ckpt_dir, self.name, which)

    def maybe_resume(self):
        path = resolve_resume(self.args.ckpt_dir, self.name, self.args.resume)
        if path is None:
            return
        which = os.path.basename(path)
        if self.ctx.is_main:
            print(f"Loading Checkpoint from {which}", flush=True)
        ck = load_checkpoint(path)
        load_model_state(self.model, ck["state_dict"])
        self.start_epoch = int(ck["epoch"]) + 1
        self.best_score = float(ck["best_score"])
        if "optimizer" in ck:
            self.optimizer.load_state_dict(ck["optimizer"])
        if "scheduler" in ck:
            self.scheduler.load_state_dict(ck["scheduler"])
        # full resume: each rank continues its own saved random streams
        self.rng_restored = restore_rank_rng(ck, self.ctx.rank, self.ctx.world_size)
        if "sampler_epoch" in ck:
            # the next epoch's DistributedSampler shuffle (seed + epoch), as the interrupted run would draw it
            self.start_epoch = int(ck["sampler_epoch"]) + 1
        self.train_sampler.set_epoch(self.start_epoch)
        if self.ctx.is_main:
            print(f"Loaded Checkpoint: {which}, with epoch {ck['epoch']} and best score {self.best_score}",
                  flush=True)

    def fit(self):
        a = self.args
        self.maybe_resume()
        log = self.log
        history = []
        for epoch in range(self.start_epoch, a.epochs):
            self.train_sampler.set_epoch(epoch)
            train_loss = self.train_epoch(epoch)
            self.scheduler.step()
            if self.dev.type == "cuda":
                torch.cuda.empty_cache()
            val_acc = self.val_epoch(epoch)
            improved = val_acc > self.best_score
            if improved:
                self.best_score = val_acc
            save_latest = bool(a.latest_every) and epoch % a.latest_every == 0
            rng_ranks = gather_rng_states() if save_latest else None  # collective: every rank's streams
            if self.ctx.is_main:
                if improved:
                    print(f"Model improved to {val_acc} so storing checkpoint", flush=True)
                    save_checkpoint(self.ckpt_path(BEST), self.model, epoch, val_acc)
                if save_latest:
                    save_checkpoint(self.ckpt_path(LATEST), self.model, epoch, self.best_score,
                                    self.optimizer, self.scheduler, rng_ranks=rng_ranks)
            rec = dict(epoch=epoch, train_loss=train_loss, val_acc=val_acc, best=self.best_score,
                       lr=self.optimizer.param_groups[0]["lr"])
            history.append(rec)
            log.log(kind="epoch", **rec)
            if not math.isfinite(train_loss):
                raise FloatingPointError(f"non-finite training loss at epoch {epoch}")
        if self._prof:  # run ended inside the profiling window
            self.global_step = a.profile_start + a.profile_steps
            self._profile_tick()
        return history
