"""Step-phase timers (HIP events) and a rank-0 JSONL metrics sink.

The reference's only throughput signal is tqdm's it/s on rank 0 (train.py:39-42).
Here every phase (data, forward, backward, comm-wait, optimizer) can be timed
with device events that are read back only at log time, so timing adds no host
syncs to the step.
"""
from __future__ import annotations

import json
import os
import time

import torch


class PhaseTimer:
    """``mark(name)`` closes the interval that started at the previous mark and books it under
    ``name``.  GPU: HIP events, read back only in ``flush`` (one sync per log interval).  CPU: host
    clock.  ``flush`` returns {phase: total ms} accumulated since the last ``reset``."""

    def __init__(self, enabled: bool, device: torch.device):
        self.enabled = enabled
        self.gpu = device.type == "cuda"
        self.events: list = []
        self.totals: dict[str, float] = {}

    def mark(self, name: str) -> None:
        if not self.enabled:
            return
        if self.gpu and torch.cuda.is_current_stream_capturing():
            return  # a replayed HIP graph is one opaque phase (the "data" mark brackets it)
        if self.gpu:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
        else:
            ev = time.perf_counter()
        self.events.append((name, ev))

    def flush(self) -> dict:
        if not self.enabled or len(self.events) < 2:
            return self.totals
        if self.gpu:
            self.events[-1][1].synchronize()
        for (_n0, e0), (n1, e1) in zip(self.events[:-1], self.events[1:]):
            dt = e0.elapsed_time(e1) if self.gpu else (e1 - e0) * 1e3
            self.totals[n1] = self.totals.get(n1, 0.0) + dt
        self.events = self.events[-1:]  # the last mark opens the next interval
        return self.totals

    def reset(self) -> None:
        self.totals = {}
        self.events = self.events[-1:]


class JsonlLogger:
    def __init__(self, path: str | None, enabled: bool):
        self.enabled = enabled and path is not None
        self.path = path
        if self.enabled:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def log(self, **kw) -> None:
        if not self.enabled:
            return
        kw.setdefault("time", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(kw) + "\n")
