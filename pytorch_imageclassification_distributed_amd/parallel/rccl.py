"""Native RCCL communicator: ``csrc/rccl_comm.cpp`` drives librccl from C++.

torch.distributed's ``nccl`` backend (ProcessGroupNCCL) runs every collective on its own internal stream
behind an event wait and hands back a ``Work`` object.  Here the collective is enqueued on a stream the
caller chooses and nothing else happens: the gradient reducer (``GradReducer(comm="rccl")``) issues each
bucket on one dedicated high-priority comm stream right behind the weight-gradient side stream, and the
compute stream waits for that stream once, before the optimizer.

Rendezvous reuses the process group's TCPStore (env:// / torchrun compatible): rank 0 creates the
``ncclUniqueId``, publishes it under a per-communicator key, every rank reads it and calls
``ncclCommInitRank`` on its device.  The library is the RCCL torch already loaded (its bundled
``librccl.so``), so the process holds one RCCL whichever side calls it.

Failure detection: ``check()`` polls ``ncclCommGetAsyncError`` (a dead peer / link error) and raises;
``close(abort=True)`` tears the communicator down without waiting for peers.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

_OPS = {"sum": 0, "max": 1, "min": 2, "prod": 3}
_SEQ = [0]  # communicators created by this process (store keys must not repeat)


def _lib():
    from .. import _ext
    C = _ext.load()
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    C.rccl_load(path if os.path.exists(path) else "librccl.so")
    return C


class RcclComm:
    """One RCCL communicator over the ranks of ``group`` (default: the world) on ``device``."""

    def __init__(self, group=None, device: torch.device | None = None):
        if not dist.is_initialized():
            raise RuntimeError("RcclComm: init the process group first (the rendezvous uses its store)")
        self.C = _lib()
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        ranks = dist.get_process_group_ranks(group) if group is not None else list(range(self.world))
        store = dist.distributed_c10d._get_default_store()
        key = f"imgcls/rccl_uid/{_SEQ[0]}/{'-'.join(map(str, ranks))}"
        _SEQ[0] += 1
        if self.rank == 0:
            store.set(key, self.C.rccl_unique_id())
        uid = store.get(key)  # blocks until rank 0 has published it
        with torch.cuda.device(self.device):
            self.handle = self.C.rccl_comm_init(bytes(uid), self.world, self.rank, self.device.index)
            # collectives run on their own stream, above the compute streams' priority
            self.stream = torch.cuda.Stream(device=self.device, priority=-1)

    # ------------------------------------------------------------------ collectives
    def all_reduce_(self, t: torch.Tensor, op: str = "sum", after: torch.cuda.Stream | None = None) -> torch.Tensor:
        """In-place all-reduce of ``t`` on the comm stream, ordered after ``after`` (default: the current
        stream).  Returns at once; ``join()`` orders a stream behind every collective issued so far."""
        self.stream.wait_stream(after if after is not None else torch.cuda.current_stream(self.device))
        self.C.rccl_all_reduce(self.handle, t, _OPS[op], self.stream.cuda_stream)
        t.record_stream(self.stream)
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0, after: torch.cuda.Stream | None = None) -> torch.Tensor:
        self.stream.wait_stream(after if after is not None else torch.cuda.current_stream(self.device))
        self.C.rccl_broadcast(self.handle, t, root, self.stream.cuda_stream)
        t.record_stream(self.stream)
        return t

    def join(self, stream: torch.cuda.Stream | None = None) -> None:
        """Make ``stream`` (default: current) wait for every collective issued so far (no host sync)."""
        (stream if stream is not None else torch.cuda.current_stream(self.device)).wait_stream(self.stream)

    # ------------------------------------------------------------------ health / teardown
    def check(self) -> None:
        """Raise if RCCL reported an asynchronous error on this communicator (peer failure)."""
        e = self.C.rccl_async_error(self.handle)
        if e != 0:
            raise RuntimeError(f"RCCL communicator error {e}: {self.C.rccl_last_error()}")

    def close(self, abort: bool = False) -> None:
        if getattr(self, "handle", 0):
            self.C.rccl_comm_close(self.handle, abort)
            self.handle = 0


def rccl_version() -> int:
    return _lib().rccl_version()
