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

import torch


class CudaPrefetcher:
    def __init__(self, loader, device: torch.device):
        self.loader = loader
        self.device = device
        self.stream = torch.cuda.Stream(device=device) if device.type == "cuda" else None

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
