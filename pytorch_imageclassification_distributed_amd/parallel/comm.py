"""Small collective helpers with the reference ``ddp_utils`` API.

* ``reduce_tensor``  - mean all-reduce of a tensor (reference ddp_utils.py:8-12).
* ``all_gather``     - all-gather of arbitrary picklable objects
                       (reference ddp_utils.py:16-56): pickle -> byte tensor ->
                       gather sizes -> pad -> gather bytes -> unpickle.  Uses
                       ``torch.frombuffer`` instead of the deprecated
                       ``ByteStorage.from_buffer`` (A17) and the group's own
                       device (RCCL: current GPU, gloo: CPU).
* ``all_reduce_sum_`` / ``all_gather_tensor`` - thin tensor paths used by the
                       metrics and SyncBN code (the object path is kept only for
                       API parity; hot paths never pickle).
"""
from __future__ import annotations

import pickle

import torch
import torch.distributed as dist


def _group_device() -> torch.device:
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def reduce_tensor(tensor: torch.Tensor) -> torch.Tensor:
    rt = tensor.clone()
    if world_size() > 1:
        dist.all_reduce(rt, op=dist.ReduceOp.SUM)
        rt /= world_size()
    return rt


def all_reduce_sum_(tensor: torch.Tensor, group=None) -> torch.Tensor:
    if world_size() > 1:
        dist.all_reduce(tensor, op=dist.ReduceOp.SUM, group=group)
    return tensor


def all_gather_tensor(tensor: torch.Tensor, group=None) -> torch.Tensor:
    """Gather equally-shaped tensors from every rank -> [world, *shape]."""
    w = dist.get_world_size(group) if dist.is_initialized() else 1
    if w == 1:
        return tensor.unsqueeze(0)
    out = torch.empty(w * tensor.numel(), dtype=tensor.dtype, device=tensor.device)
    dist.all_gather_into_tensor(out, tensor.contiguous().reshape(-1), group=group)
    return out.view((w,) + tuple(tensor.shape))


def all_gather(data):
    """Run all_gather on arbitrary picklable data; returns a list with one entry per rank."""
    ws = world_size()
    if ws == 1:
        return [data]
    dev = _group_device()
    buf = pickle.dumps(data)
    tensor = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev)
    local_size = torch.tensor([tensor.numel()], device=dev, dtype=torch.int64)
    sizes = [torch.zeros(1, device=dev, dtype=torch.int64) for _ in range(ws)]
    dist.all_gather(sizes, local_size)
    sizes = [int(s.item()) for s in sizes]
    max_size = max(sizes)
    if tensor.numel() < max_size:
        tensor = torch.cat([tensor, torch.zeros(max_size - tensor.numel(), dtype=torch.uint8, device=dev)])
    outs = [torch.empty(max_size, dtype=torch.uint8, device=dev) for _ in range(ws)]
    dist.all_gather(outs, tensor)
    return [pickle.loads(o.cpu().numpy().tobytes()[:s]) for s, o in zip(sizes, outs)]
