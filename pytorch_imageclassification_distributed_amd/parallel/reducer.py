"""Bucketed gradient all-reduce overlapped with backward (our DDP).

Reference: ``DistributedDataParallel(model, device_ids=[local_rank], ...)``
(train.py:128) - the C++ Reducer all-reduces 25 MiB gradient buckets (1 MiB
first bucket) as they become ready during backward, after broadcasting rank 0's
parameters and buffers at construction (torch/nn/parallel/distributed.py:
659-666, 828-871, 1197-1248).

MI355X design:
* every gradient lives in ONE flat fp32 buffer laid out in bucket order, so a
  bucket is a contiguous slice (one RCCL call, no pack/unpack) and the fused
  Adam kernel reads gradients in place;
* the flat buffer is a ``GradArena``: our backward kernels write each gradient
  straight into its slot (``ops.grad_arena``), so the ``post_accumulate_grad``
  hook only copies gradients produced elsewhere (ATen ops), and, when the bucket's last gradient lands, launches an
  *asynchronous* RCCL all-reduce.  ProcessGroupNCCL runs it on its own HIP
  stream after an event wait on the compute stream, so the reduction of early
  buckets overlaps the rest of backward; ``finish()`` makes the compute stream
  wait for the comm stream (no host sync);
* buckets are re-laid-out once, after the first backward, in the order the
  gradients actually became ready (DDP's bucket rebuild);
* the 1/world mean is *not* applied as a separate pass: ``grad_scale`` is handed
  to the fused optimizer (Adam is scale-invariant only up to eps, so the scale
  is applied exactly, not skipped);
* bucket size defaults to 32 MiB: on MI355X each GPU has 7 xGMI links of
  ~153 GB/s; RCCL's ring/tree algorithms saturate them from a few MiB, and
  fewer, larger buckets mean fewer ~10-20 us collective launches.  The first
  bucket is kept small (1 MiB) so communication starts early in backward.
* the LAST bucket is cut into pieces of at most ``tail_bucket_mb`` (4 MiB): its gradients (ResNet's layer1
  and stem, ~28 MiB) are the last ones backward produces, so a whole-bucket collective could only start
  after the weight-gradient side stream drained and would sit entirely after backward; pieces launch as
  their own gradients land, and only the final few MiB stay exposed (``ms_comm_wait`` in bench.py's line).
* optional bf16 gradient transport (``comm_dtype=torch.bfloat16``) halves the
  xGMI bytes.
* ``comm="rccl"``: the buckets go through our own C++ RCCL communicator
  (``parallel/rccl.py``) instead of ProcessGroupNCCL - each collective is enqueued
  on one dedicated high-priority comm stream straight behind the weight-gradient
  side stream (no Work objects, no per-collective event bookkeeping), and
  ``finish()`` is a single stream wait.
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.distributed as dist
import torch.nn as nn

from ..ops.grad_arena import GradArena
from . import comm_timer

# 1: with the native communicator, a captured whole-step HIP graph carries the bucket collectives themselves
# (forked onto the comm stream inside the graph, overlapping the rest of the captured backward); 0: the
# capture defers them and one flat all-reduce runs after every replay
GRAPH_COLLECTIVES = os.environ.get("IMGCLS_GRAPH_COLLECTIVES", "1") == "1"


def _comm_stream(dev):
    """The HIP path's side stream for a bucket all-reduce (ops.hip.comm_stream), else None."""
    if dev.type != "cuda":
        return None
    from ..ops import hip
    return hip.comm_stream(dev)


def broadcast_module_state(module: nn.Module, src: int = 0, group=None) -> None:
    """Coalesced broadcast of parameters and buffers from ``src`` (DDP ctor, X2)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    tensors = [t for t in module.state_dict().values() if isinstance(t, torch.Tensor)]
    by_dtype: dict = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (_dt, _dev), ts in by_dtype.items():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        dist.broadcast(flat, src, group=group)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n


class GradReducer:
    def __init__(self, module: nn.Module, group=None, bucket_cap_mb: float = 32.0,
                 first_bucket_mb: float = 1.0, broadcast: bool = True,
                 rebuild_buckets: bool = True, comm_dtype: torch.dtype | None = None, comm: str = "pg",
                 force_collectives: bool = False, timeout_s: float = 600.0, tail_bucket_mb: float = 4.0):
        self.module = module
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.params = [p for p in module.parameters() if p.requires_grad]
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.bucket_cap = int(bucket_cap_mb * 2**20) // 4
        self.first_cap = int(first_bucket_mb * 2**20) // 4
        self.tail_cap = int(tail_bucket_mb * 2**20) // 4 if tail_bucket_mb > 0 else 0
        self.comm_dtype = comm_dtype
        self._rebuild_pending = rebuild_buckets and self.world > 1
        self._ready_order: list[int] = []
        self.works: list = []
        self.arena: GradArena | None = None
        # force_collectives (tests): run the bucket collectives even in a world of one
        self._collect = self.world > 1 or force_collectives
        # diagnostic only (never a benchmark: bench.py relabels its line): no gradient collective at all, to time
        # a multi-rank step without its gradient all-reduce (ranks sharing one GPU over gloo, where that
        # all-reduce is a host copy that swamps everything else)
        if os.environ.get("IMGCLS_DIAG_SKIP_GRAD_COMM", "0") == "1":
            self._collect = False
        self.rccl = None
        self.watchdog = None
        # deferred (whole-step HIP-graph replay at N > 1): backward only fills the arena; no collective is
        # issued from a hook (a gloo / process-group call cannot sit inside a captured graph), and
        # ``flat_all_reduce`` sums the whole arena once after the replay
        self.deferred = False
        if comm == "rccl" and self._collect:
            from .rccl import CommWatchdog, RcclComm
            dev = next(iter(self.params)).device
            self.rccl = RcclComm(group, dev)
            # the process group's timeout / async error handling do not watch this communicator
            self.watchdog = CommWatchdog(self.rccl.async_error, lambda: self.rccl.close(abort=True), timeout_s)
        elif comm not in ("pg", "rccl"):
            raise ValueError(f"GradReducer: comm must be 'pg' or 'rccl', not {comm!r}")
        self._verify_param_shapes()
        if broadcast:
            broadcast_module_state(module, 0, group)
        self._build(list(reversed(range(len(self.params)))))
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    def _verify_param_shapes(self) -> None:
        """DDP's ``_verify_param_shape_across_processes`` (X1, torch/nn/parallel/distributed.py:862): every
        rank must hold the same parameter list, or the flat-buffer buckets would pair different tensors."""
        if self.world == 1:
            return
        mine = [(tuple(p.shape), str(p.dtype)) for p in self.params]
        allp = [None] * self.world
        dist.all_gather_object(allp, mine, group=self.group)
        for r, theirs in enumerate(allp):
            if theirs != mine:
                bad = next((i for i, (a, b) in enumerate(zip(mine, theirs)) if a != b), min(len(mine), len(theirs)))
                raise RuntimeError(
                    f"GradReducer: parameter list differs between this rank and rank {r} "
                    f"({len(mine)} vs {len(theirs)} tensors; first mismatch at index {bad}: "
                    f"{mine[bad] if bad < len(mine) else None} vs {theirs[bad] if bad < len(theirs) else None})")

    # ------------------------------------------------------------------ layout
    def _build(self, order: list[int]) -> None:
        if self.arena is None:
            self.arena = GradArena(self.params, order)
        else:
            self.arena.layout(order)
        offsets = self.arena.offsets
        buckets, cur, cur_start = [], [], 0
        cap = self.first_cap
        for i in order:
            off = offsets[i]
            if cur and off - cur_start + self.params[i].numel() > cap:
                buckets.append((cur_start, off, cur))
                cur, cur_start, cap = [], off, self.bucket_cap
            cur.append(i)
        if cur:
            buckets.append((cur_start, self.arena.flat.numel(), cur))
        if self.tail_cap and len(buckets) > 1 and buckets[-1][1] - buckets[-1][0] > self.tail_cap:
            buckets = buckets[:-1] + self._split(buckets[-1], offsets)
        self.buckets = buckets
        self.bucket_of = [0] * len(self.params)
        for b, (_s, _e, idx) in enumerate(buckets):
            for i in idx:
                self.bucket_of[i] = b
        self._reset_counts()

    def _split(self, bucket, offsets) -> list:
        """Cut the last bucket into pieces of at most ``tail_cap`` elements on parameter boundaries (a single
        larger parameter keeps a piece of its own), in the same ready order."""
        start, end, idx = bucket
        out, cur, cur_start = [], [], start
        for i in idx:
            off = offsets[i]
            if cur and off - cur_start + self.params[i].numel() > self.tail_cap:
                out.append((cur_start, off, cur))
                cur, cur_start = [], off
            cur.append(i)
        out.append((cur_start, end, cur))
        return out

    @property
    def flat(self) -> torch.Tensor:
        return self.arena.flat

    def begin(self) -> None:
        """Zero and arm the gradient slots before a backward (one memset)."""
        self.arena.begin()

    def _reset_counts(self) -> None:
        self.pending = [len(idx) for (_s, _e, idx) in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.got = [False] * len(self.params)

    def bucket_sizes_mb(self) -> list[float]:
        return [(e - s) * 4 / 2**20 for (s, e, _i) in self.buckets]

    # ------------------------------------------------------------------ hooks
    @torch.no_grad()
    def _on_grad(self, p: torch.Tensor) -> None:
        i = self.index[id(p)]
        if not self.arena.owns(p):
            v = self.arena.view(i)
            v.copy_(p.grad)
            p.grad = v
        if self._rebuild_pending:
            self._ready_order.append(i)
        if not self.got[i]:
            self.got[i] = True
            b = self.bucket_of[i]
            self.pending[b] -= 1
            if self.pending[b] == 0:
                self._launch(b)

    def _launch(self, b: int) -> None:
        self.launched[b] = True
        if not self._collect or self.deferred:
            return
        s, e, _ = self.buckets[b]
        t = self.flat[s:e]
        # weight gradients may still be in flight on the HIP path's side stream: issue the collective
        # from that stream once it has waited for the compute stream (ProcessGroupNCCL orders its RCCL
        # stream behind the current one), so it follows the bucket's gradients from both streams
        side = _comm_stream(t.device)
        main = torch.cuda.current_stream(t.device) if side is not None else None
        if comm_timer.active() and t.is_cuda:
            comm_timer.mark("first_bucket", side if side is not None else torch.cuda.current_stream(t.device))
        if self.rccl is not None:
            after = side if side is not None else torch.cuda.current_stream(t.device)
            with torch.cuda.stream(after):
                c = t.to(self.comm_dtype) if self.comm_dtype not in (None, torch.float32) else t
            self.rccl.all_reduce_(c, after=after)
            self.works.append((None, t, c) if c is not t else (None, None, None))
            return
        with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
            if self.comm_dtype is not None and self.comm_dtype != torch.float32:
                c = t.to(self.comm_dtype)
                if main is not None:
                    c.record_stream(main)  # copied back on the compute stream in finish()
                self.works.append((dist.all_reduce(c, group=self.group, async_op=True), t, c))
            else:
                self.works.append((dist.all_reduce(t, group=self.group, async_op=True), None, None))

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def finish(self) -> float:
        """Flush the remaining buckets, make the compute stream wait for RCCL.

        Returns the factor that turns the summed gradients into the world mean
        (consumed by the fused optimizer).
        """
        for i, p in enumerate(self.params):  # parameters that got no gradient
            if not self.got[i]:
                v = self.arena.view(i)
                v.zero_()
                p.grad = v
                self.got[i] = True
                b = self.bucket_of[i]
                self.pending[b] -= 1
        timed = comm_timer.active() and self.flat.is_cuda
        if timed:  # (no side stream: backward ended on this stream, nothing lags behind it)
            comm_timer.mark("compute_end")
            comm_timer.mark("side_joined")
        for b in range(len(self.buckets)):
            if not self.launched[b]:
                self._launch(b)
        if self.rccl is not None and self.works:
            self.rccl.join()  # the compute stream waits for every bucket's collective
            if not torch.cuda.is_current_stream_capturing():  # a captured step is armed after each replay
                self.arm_watchdog(self.rccl.stream)
        for work, dst, comp in self.works:
            if work is not None:
                work.wait()
            if dst is not None:
                dst.copy_(comp)
        self.works.clear()
        if timed:
            comm_timer.mark("comm_end")
        self._reset_counts()
        if self._rebuild_pending:
            self._rebuild_pending = False
            seen = set(self._ready_order)
            order = self._ready_order + [i for i in reversed(range(len(self.params))) if i not in seen]
            if self.world > 1:
                # every rank must lay out the same buckets (a bucket is one collective): take rank 0's
                # observed order, as DDP's bucket rebuild does (sync_bucket_indices)
                box = [order]
                dist.broadcast_object_list(box, src=dist.get_global_rank(self.group, 0) if self.group else 0,
                                           group=self.group)
                order = box[0]
            self._build(order)
            self._ready_order = []
        return 1.0 / self.world

    def reset_after_capture(self) -> None:
        """Forget the hook bookkeeping of a captured backward (the replays do not run the hooks)."""
        for p in self.params:  # the slots stay the gradients' storage (the captured kernels write there)
            p.grad = self.arena.view(self.index[id(p)])
        self._reset_counts()

    @property
    def graph_collectives(self) -> bool:
        """The bucket collectives can sit inside a captured whole-step graph: they go through our own RCCL
        communicator, enqueued on its comm stream (a forked branch of the capture that joins back before the
        optimizer), with no Work object and no host wait.  ProcessGroupNCCL's Work / watchdog bookkeeping is
        not capture-safe, so the process-group path stays ``deferred`` (``flat_all_reduce`` after replay)."""
        return self.rccl is not None and self._collect and GRAPH_COLLECTIVES

    def arm_watchdog(self, stream) -> None:
        """Register "every collective enqueued so far on ``stream`` has finished" with the CommWatchdog: a step
        whose collectives never complete ends the process instead of hanging (native communicator only)."""
        if self.watchdog is not None:
            done = torch.cuda.Event()
            done.record(stream)
            self.watchdog.arm(done)

    @torch.no_grad()
    def flat_all_reduce(self) -> float:
        """After a replayed backward (``deferred``): one all-reduce of the whole gradient arena on the current
        stream, in place of the per-bucket collectives, in the same transport dtype as the bucketed path
        (``comm_dtype``: bf16 casts, reduces and copies back).  Returns the mean factor for the optimizer."""
        if self._collect:
            t = self.flat
            c = t.to(self.comm_dtype) if self.comm_dtype not in (None, torch.float32) else t
            if self.rccl is not None:
                self.rccl.all_reduce_(c)
                self.rccl.join()
                self.arm_watchdog(self.rccl.stream)
            else:
                dist.all_reduce(c, group=self.group)
            if c is not t:
                t.copy_(c)
        return 1.0 / self.world

    def average_(self) -> None:
        """Turn the summed flat gradients into means in place (for stock optimizers)."""
        if self.world > 1:
            self.flat.mul_(1.0 / self.world)

    def sync_buffers(self, src: int = 0) -> None:
        """DDP ``broadcast_buffers`` (X3): redundant with SyncBN, kept for parity."""
        if self.world == 1:
            return
        for b in self.module.buffers():
            dist.broadcast(b, src, group=self.group)

    def check(self) -> None:
        """Raise if the native communicator reported an asynchronous error (log-interval health check)."""
        if self.rccl is not None:
            self.rccl.check()

    def close(self) -> None:
        """Stop the watchdog and free the native communicator (no-op on the process-group path)."""
        if self.watchdog is not None:
            self.watchdog.stop()
            self.watchdog = None
        if self.rccl is not None:
            self.rccl.close()
            self.rccl = None

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        self.arena.detach_params()
