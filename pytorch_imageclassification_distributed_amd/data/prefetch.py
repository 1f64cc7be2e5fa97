"""Host->device double buffering on a dedicated copy stream.

Reference: the DataLoader pins batches (``pin_memory=True``, train.py:114) and
the loop issues ``.cuda(non_blocking=True)`` on the compute stream
(train.py:45-46), so the copy of batch i+1 cannot start before batch i's
kernels are enqueued behind it.  Here batch i+1's pinned-memory
``hipMemcpyAsync`` is issued on a separate HIP stream while batch i computes;
the compute stream waits on an event, and ``record_stream`` keeps the caching
allocator from recycling the buffer early.
"""
from __future__ import annotations

import os

import torch

# IMGCLS_COPY_STREAM: "high" (highest priority, default) | "default" (a normal-priority pool stream) | "low"
COPY_STREAM = os.environ.get("IMGCLS_COPY_STREAM", "high")


def copy_stream(device) -> torch.cuda.Stream:
    """The stream a loader issues its host->device copies (and input conversion) on.

    High priority by default.  With GPU_MAX_HW_QUEUES=4 (HIP's default) the normal-priority pool streams
    share hardware queues, and the copy stream landed on the weight-gradient side stream's queue: each
    batch's 154 MB H2D copy then waited behind the step's last wgrad and the next step waited for the
    copy - 2.9 ms of idle GPU per ResNet-50 b1024 step (rocprofv3 timeline, profiles/r9o_host_copy_queue.txt).
    On its own high-priority queue the copy overlaps the step: --data host 14000 vs --data device 13977
    img/s on one box (was 13385)."""
    if COPY_STREAM == "high":
        return torch.cuda.Stream(device=device, priority=torch.cuda.Stream.priority_range()[1])
    if COPY_STREAM == "low":
        return torch.cuda.Stream(device=device, priority=torch.cuda.Stream.priority_range()[0])
    return torch.cuda.Stream(device=device)


class CudaPrefetcher:
    def __init__(self, loader, device: torch.device):
        self.loader = loader
        self.device = device
        self.stream = copy_stream(device) if device.type == "cuda" else None

    def __len__(self):
        return len(self.loader)

    def _to_device(self, batch):
        out = {}
        for k, v in batch.items():
            if isinstance(v, torch.Tensor):
                out[k] = v.to(self.device, non_blocking=True)
            else:
                out[k] = v
        return out

    def __iter__(self):
        it = iter(self.loader)
        if self.stream is None:
            for b in it:
                yield b
            return
        nxt = None
        try:
            first = next(it)
        except StopIteration:
            return
        with torch.cuda.stream(self.stream):
            nxt = self._to_device(first)
        while nxt is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            cur = nxt
            for v in cur.values():
                if isinstance(v, torch.Tensor) and v.is_cuda:
                    v.record_stream(torch.cuda.current_stream(self.device))
            try:
                b = next(it)
                with torch.cuda.stream(self.stream):
                    nxt = self._to_device(b)
            except StopIteration:
                nxt = None
            yield cur
