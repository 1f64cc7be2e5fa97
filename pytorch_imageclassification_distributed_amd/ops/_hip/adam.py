"""Fused Adam: the per-step pointer table and the single-launch update (shadows refreshed in the same pass).

Split out of ``ops/hip.py`` (the facade that re-exports every name here).
"""
from __future__ import annotations

import numpy as np
import torch

from . import shadows as _shadows
from .common import C, CL, _upload
from .shadows import (_mx_tiles, shadow_for_optimizer, shadow_generation, shadow_mx_for_optimizer,
                      shadow_t_for_optimizer)


# ---------------------------------------------------------------------------
# fused Adam
# ---------------------------------------------------------------------------
_ADAM_CHUNK = 65536
_TENSOR_DT = np.dtype([("p", "<u8"), ("g", "<u8"), ("m", "<u8"), ("v", "<u8"), ("s", "<u8"), ("n", "<i8")])
_WTJOB_DT = np.dtype([("w", "<u8"), ("o", "<u8"), ("co", "<i4"), ("t", "<i4"), ("ci", "<i4"), ("pad", "<i4")])


def _same_memory_order(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Dense tensors whose elements sit in the same order in memory (size-1 dims ignored)."""
    if a.shape != b.shape:
        return False
    dense = lambda t: t.is_contiguous() or t.is_contiguous(memory_format=CL)  # noqa: E731
    if not (dense(a) and dense(b)):
        return False
    return all(sa == sb for n, sa, sb in zip(a.shape, a.stride(), b.stride()) if n > 1)


def adam_build_table(opt, items):
    if C.weight_t_job_bytes() != _WTJOB_DT.itemsize:
        raise RuntimeError("weight_t_tiles: job record layout mismatch between Python and the kernel")
    groups = {}
    wt_jobs = []
    mx_jobs = []
    for gi, group, p in items:
        groups.setdefault(gi, (group, []))[1].append(p)
    tables = []
    for gi, (group, ps) in sorted(groups.items()):
        recs = np.zeros(len(ps), dtype=_TENSOR_DT)
        chunks = []
        for t, p in enumerate(ps):
            st = opt.state[p]
            sh = shadow_for_optimizer(p)
            recs[t] = (p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(),
                       sh.data_ptr() if sh is not None else 0, p.numel())
            stt = shadow_t_for_optimizer(p) if sh is not None else None
            if stt is not None:
                wt_jobs.append((sh.data_ptr(), stt[0].data_ptr()) + tuple(stt[1:]) + (0,))
            smx = shadow_mx_for_optimizer(p) if sh is not None else None
            if smx is not None:
                mx_jobs.append((p.data_ptr(), smx[0].data_ptr(), smx[1].data_ptr(), p.numel()))
            for ck in range(-(-p.numel() // _ADAM_CHUNK)):
                chunks.append((t, ck))
            if not _same_memory_order(p, p.grad):
                raise RuntimeError("fused Adam: gradient layout differs from parameter layout")
        dev = ps[0].device
        tab = _upload(recs.view(np.uint8).copy(), dev)
        ck = _upload(np.asarray(chunks, dtype=np.int32).reshape(-1), dev)
        lr_step = getattr(opt, "_lr_step", {}).get(gi)
        if lr_step is None:
            step0 = float(opt.state[ps[0]]["step"]) if "step" in opt.state[ps[0]] else 0.0
            lr_step = torch.tensor([group["lr"], step0], dtype=torch.float32, device=dev)
            opt.__dict__.setdefault("_lr_step", {})[gi] = lr_step
        tables.append((gi, tab, ck, len(chunks), lr_step, [p for p in ps]))
    wt = None
    if wt_jobs:
        jobs = np.array(wt_jobs, dtype=_WTJOB_DT)
        tiles = [(j, t, co0, ci0) for j, (_w, _o, co, taps, ci, _p) in enumerate(wt_jobs)
                 for t in range(taps) for co0 in range(0, co, 64) for ci0 in range(0, ci, 64)]
        wt = (_upload(jobs.view(np.uint8).copy(), tables[0][1].device),
              _upload(np.asarray(tiles, dtype=np.int32).reshape(-1), tables[0][1].device), len(tiles))
    mx = None
    if mx_jobs:
        dev0 = tables[0][1].device
        tiles = _mx_tiles(mx_jobs)
        mx = (_upload(np.array(mx_jobs, dtype=_shadows._MXW_DT).view(np.uint8).copy(), dev0),
              _upload(np.asarray(tiles, dtype=np.int32).reshape(-1), dev0), len(tiles))
    return (tables, shadow_generation(), wt, mx)


def adam_step(opt, items, table, grad_scale):
    tables, gen, wt, mx = table
    if gen != shadow_generation():
        opt._table_key = None  # rebuild next step so new shadows are kept fresh
    for gi, tab, ck, nck, lr_step, ps in tables:
        group = opt.param_groups[gi]
        b1, b2 = group["betas"]
        C.adam_tick(lr_step, float(group["lr"]))
        C.adam(tab, ck, nck, lr_step, b1, b2, group["eps"], group["weight_decay"], float(grad_scale), _ADAM_CHUNK)
    if wt is not None:  # refresh every transposed dgrad shadow from the updated KRSC shadows: one launch
        C.weight_t_tiles(*wt)
    if mx is not None:  # and every MX-FP8 forward copy from the updated fp32 masters: one launch
        C.mx_quant_w(*mx)
    opt._host_steps = getattr(opt, "_host_steps", 0) + 1


# names this part owns (ops/hip.py re-exports them)
_OWNED = (
    '_ADAM_CHUNK', '_TENSOR_DT', '_WTJOB_DT', '_same_memory_order', 'adam_build_table', 'adam_step',
)
