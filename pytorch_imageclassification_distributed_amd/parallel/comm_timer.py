"""Per-step communication timeline on the GPU clock (bench.py at N > 1, ``--comm-timing``).

Device events mark, per training step, on the streams where things happen:

* ``first_bucket``  - the first gradient bucket's all-reduce is issued (its stream, parallel/reducer.py);
* ``compute_end``   - the compute stream finished backward (ops/hip.py ``join_side_streams``, before it
                      waits for the weight-gradient side stream);
* ``side_joined``   - the compute stream has caught up with the side stream (the last weight gradients);
* ``comm_end``      - every bucket all-reduce has completed (reducer ``finish``, after the waits);
* ``step_start`` / ``step_end`` - the trainer brackets the step;
* spans ``syncbn_fwd`` / ``syncbn_bwd`` - every SyncBN statistics exchange (the one-shot peer kernel, or
  the RCCL all-reduce with its reduce / finalize kernels), summed per step.

``summary()`` (one device sync, after the timed loop) turns them into the numbers an N > 1 run needs to
be read: how long before the end of backward the first collective could start (overlap window), how
long the compute stream waited for the lagging weight gradients, and how much collective time stayed
exposed after both.  Nothing here runs unless a timer is installed (``install``).
"""
from __future__ import annotations

import contextlib

import torch

_TIMER = None


class StepCommTimer:
    def __init__(self):
        self.steps: list[dict] = []
        self.cur: dict | None = None
        self.spans: list[dict] = []  # per step: name -> [(start, end)]
        self.cur_spans: dict | None = None

    def begin(self, stream=None) -> None:
        self.cur = {}
        self.cur_spans = {}
        self.mark("step_start", stream)

    @contextlib.contextmanager
    def span(self, name: str, stream=None):
        """Time the work enqueued inside the block on ``stream`` (default: current); summed per step."""
        if self.cur_spans is None:
            yield
            return
        st = stream if stream is not None else torch.cuda.current_stream()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        try:
            yield
        finally:
            b.record(st)
            self.cur_spans.setdefault(name, []).append((a, b))

    def mark(self, name: str, stream=None) -> None:
        if self.cur is None or name in self.cur:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream if stream is not None else torch.cuda.current_stream())
        self.cur[name] = e

    def end(self, stream=None) -> None:
        if self.cur is None:
            return
        self.mark("step_end", stream)
        self.steps.append(self.cur)
        self.spans.append(self.cur_spans or {})
        self.cur = None
        self.cur_spans = None

    def summary(self) -> dict:
        """Mean milliseconds over the recorded steps (syncs the device once)."""
        torch.cuda.synchronize()
        acc: dict = {}

        def add(key, a, b, st):
            if a in st and b in st:
                acc.setdefault(key, []).append(st[a].elapsed_time(st[b]))

        for st in self.steps:
            add("ms_step_gpu", "step_start", "step_end", st)
            add("ms_first_bucket_before_bwd_end", "first_bucket", "compute_end", st)
            add("ms_side_stream_tail", "compute_end", "side_joined", st)
            add("ms_comm_wait", "side_joined", "comm_end", st)
        for sp in self.spans:
            for name, pairs in sp.items():
                acc.setdefault(f"ms_{name}", []).append(sum(a.elapsed_time(b) for a, b in pairs))
                acc.setdefault(f"n_{name}", []).append(len(pairs))
        return {k: round(sum(v) / len(v), 3) for k, v in acc.items() if v}


def install() -> StepCommTimer:
    global _TIMER
    _TIMER = StepCommTimer()
    return _TIMER


def uninstall() -> None:
    global _TIMER
    _TIMER = None


def mark(name: str, stream=None) -> None:
    if _TIMER is not None:
        _TIMER.mark(name, stream)


def active() -> bool:
    return _TIMER is not None


def span(name: str, stream=None):
    """Context manager timing the enclosed device work into the installed timer's ``ms_<name>``."""
    return _TIMER.span(name, stream) if _TIMER is not None else contextlib.nullcontext()
