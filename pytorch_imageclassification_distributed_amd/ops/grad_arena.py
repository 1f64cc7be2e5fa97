"""Persistent flat gradient storage (replaces per-step ``torch.zeros`` for every ``.grad``).

The reference lets autograd allocate a fresh gradient per parameter per step and
DDP's C++ Reducer copy it into a bucket (torch/csrc/distributed/c10d/reducer.cpp,
"gradient_as_bucket_view" off by default; reference train.py:128).  On MI355X
that is ~160 zero-fill/copy launches per step and, worse, gradient pointers
that change every step, which forces the fused optimizer to re-upload its
pointer table (a host-synchronous copy).

``GradArena`` owns ONE fp32 buffer laid out in a caller-chosen order (the
reducer's bucket order, so a bucket is a contiguous slice).  ``begin()`` zeroes
it with a single memset and "arms" every slot; a backward kernel asks for its
output with :func:`grad_buffer` and receives a fresh strided view of its slot
(matching the parameter's layout), which autograd adopts as ``param.grad``
without a copy.  A slot is handed out at most once per ``begin()``: a second
contribution (gradient accumulation, a parameter used twice) gets an ordinary
tensor and autograd accumulates into the slot in place, so semantics never
change - only the allocations disappear.
"""
from __future__ import annotations

import torch

ALIGN = 64  # elements (256 B): every slot starts on a cache-line boundary


class GradArena:
    def __init__(self, params, order=None):
        self.params = list(params)
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.flat = None
        self.offsets = [0] * len(self.params)
        self.handed = [True] * len(self.params)  # nothing armed until begin()
        self.layout(order if order is not None else list(range(len(self.params))))
        for p in self.params:
            p._imgcls_arena = self

    def layout(self, order):
        """(Re)lay the slots out in ``order``; live gradients are moved to the new slots."""
        old_flat, old_off = self.flat, list(self.offsets)
        off = 0
        for i in order:
            self.offsets[i] = off
            off += (self.params[i].numel() + ALIGN - 1) // ALIGN * ALIGN
        dev = self.params[0].device
        self.flat = torch.zeros(max(off, 1), dtype=torch.float32, device=dev)
        if old_flat is not None:
            with torch.no_grad():
                for i, p in enumerate(self.params):
                    if p.grad is not None and self.owns(p, old_flat, old_off[i]):
                        v = self.view(i)
                        v.copy_(p.grad)
                        p.grad = v
        return off

    def owns(self, p, flat=None, off=None) -> bool:
        """True when ``p.grad`` currently aliases its slot."""
        i = self.index[id(p)]
        flat = self.flat if flat is None else flat
        off = self.offsets[i] if off is None else off
        g = p.grad
        return (g is not None and g.data_ptr() == flat.data_ptr() + 4 * off
                and g.stride() == p.stride() and g.dtype == torch.float32)

    def view(self, i: int) -> torch.Tensor:
        p = self.params[i]
        return torch.as_strided(self.flat, p.size(), p.stride(), self.offsets[i])

    def begin(self) -> None:
        """Zero every slot (one memset) and arm them for the next backward."""
        self.flat.zero_()
        self.handed = [False] * len(self.params)

    def take(self, p):
        i = self.index.get(id(p))
        if i is None or self.handed[i] or p.grad is not None:
            return None
        self.handed[i] = True
        return self.view(i)

    def detach_params(self) -> None:
        for p in self.params:
            if getattr(p, "_imgcls_arena", None) is self:
                del p._imgcls_arena


def arena_slot(p):
    """``p``'s armed arena slot (zeroed, persistent: autograd adopts it as ``p.grad`` without touching
    it), or None when ``p`` has no arena or its slot was already handed out this step."""
    a = getattr(p, "_imgcls_arena", None)
    return a.take(p) if a is not None else None


def grad_buffer(p, zero: bool = True) -> torch.Tensor:
    """Output buffer for ``p``'s gradient: its armed arena slot (already zero), else a new tensor
    with ``p``'s shape and memory layout."""
    a = getattr(p, "_imgcls_arena", None)
    if a is not None:
        v = a.take(p)
        if v is not None:
            return v
    out = torch.empty_strided(p.size(), p.stride(), dtype=torch.float32, device=p.device)
    return out.zero_() if zero else out
