"""Process-group bring-up: one process per GPU, RCCL over xGMI (or gloo on CPU).

Reference: ``dist.init_process_group('nccl', rank=args.local_rank)`` followed by
``torch.cuda.set_device`` (reference train.py:99-106).  Fixed here:
* RANK comes from the environment, LOCAL_RANK only picks the device (A8);
* the device is bound *before* the process group is created so RCCL's
  communicator binds to the right GPU (A20);
* ``--local-rank`` / ``--local_rank`` / ``LOCAL_RANK`` are all accepted (A7);
* a single process without launcher env vars still gets a (world=1) group on
  127.0.0.1, so the same code path runs everywhere.

On ROCm the ``"nccl"`` backend *is* RCCL; RCCL picks the xGMI point-to-point
links between MI355X GPUs of a node automatically.
"""
from __future__ import annotations

import datetime
import os
import socket
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistContext:
    rank: int
    world_size: int
    local_rank: int
    device: torch.device
    backend: str

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def env_local_rank(cli_local_rank: int | None = None) -> int:
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"])
    return int(cli_local_rank or 0)


def init_distributed(device: str = "auto", backend: str | None = None,
                     local_rank: int | None = None, timeout_min: float = 10.0) -> DistContext:
    """Initialise (or reuse) the default process group and bind the device."""
    lr = env_local_rank(local_rank)
    if device == "auto":
        device = "cuda" if torch.cuda.is_available() else "cpu"
    if device == "cuda":
        # one process per GPU; ranks beyond the visible devices share them (functional tests only)
        idx = lr % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(idx)
        dev = torch.device("cuda", idx)
    else:
        dev = torch.device("cpu")
    if backend is None or backend == "auto":
        backend = "nccl" if dev.type == "cuda" else "gloo"
    if backend == "rccl":
        backend = "nccl"
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(_free_port())
        rank = int(os.environ.get("RANK", "0"))
        world = int(os.environ.get("WORLD_SIZE", "1"))
        kw = {}
        if backend == "nccl":
            kw["device_id"] = dev
            # a failed / hung collective aborts the communicator and raises in every surviving rank
            # instead of hanging until the job is killed
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        dist.init_process_group(backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(minutes=timeout_min), **kw)
    return DistContext(dist.get_rank(), dist.get_world_size(), lr, dev, dist.get_backend())


def barrier(ctx: DistContext | None = None) -> None:
    if not dist.is_initialized():
        return
    if ctx is not None and ctx.backend == "nccl":
        dist.barrier(device_ids=[ctx.local_rank])
    else:
        dist.barrier()


def destroy() -> None:
    """Tear down the native RCCL communicators, the SyncBN peer channels (IPC mappings, buffers), then the
    process group."""
    from .peer import teardown_peer_syncbn
    from .rccl import close_all
    close_all()
    teardown_peer_syncbn()
    if dist.is_initialized():
        dist.destroy_process_group()


def get_world_size() -> int:
    return dist.get_world_size() if dist.is_initialized() else 1


def get_rank() -> int:
    return dist.get_rank() if dist.is_initialized() else 0
