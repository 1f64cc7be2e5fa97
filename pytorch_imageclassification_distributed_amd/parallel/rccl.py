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
``close(abort=True)`` tears the communicator down without waiting for peers.  ProcessGroupNCCL's watchdog
(``TORCH_NCCL_ASYNC_ERROR_HANDLING``, the PG timeout) does not cover this communicator, so ``CommWatchdog``
does its job: a host thread polls the async error and the age of every step's "collectives done" event,
and when either goes bad it aborts the communicator and ends the process non-zero - a dead peer cannot
leave the compute stream waiting on a comm stream that never finishes (reference: the NCCL PG timeout,
/root/reference/train.py:102).
"""
from __future__ import annotations

import collections
import os
import sys
import threading
import time

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


_LIVE: "list[RcclComm]" = []  # communicators not yet closed (parallel.dist.destroy() closes them)


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
        _LIVE.append(self)

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

    def async_error(self) -> int:
        h = getattr(self, "handle", 0)  # read once: close() may run between a check and the call
        return int(self.C.rccl_async_error(h)) if h else 0

    def close(self, abort: bool = False) -> None:
        if getattr(self, "handle", 0):
            self.C.rccl_comm_close(self.handle, abort)
            self.handle = 0
        if self in _LIVE:
            _LIVE.remove(self)


def close_all(abort: bool = False) -> None:
    """Stop every live watchdog first (a watchdog polling a communicator that is being destroyed would
    read a teardown as a fault and exit non-zero), then close every communicator."""
    for w in list(_WATCHDOGS):
        w.stop()
    for c in list(_LIVE):
        c.close(abort)


_WATCHDOGS: "list[CommWatchdog]" = []  # running watchdogs (close_all stops them before any communicator goes)


class CommWatchdog:
    """Host-side deadline for collectives on a communicator the process group does not watch.

    ``arm(done)`` registers a completion probe (a HIP event recorded on the comm stream after a step's
    collectives; anything with ``query() -> bool``).  A daemon thread polls every ``interval`` s: if
    ``poll_error()`` is non-zero, or the oldest unfinished probe is older than ``timeout`` s, it calls
    ``abort()`` (RcclComm.close(abort=True)) and ``on_fatal(message)`` - by default a message on stderr and
    ``os._exit(exit_code)``, the process-level equivalent of ProcessGroupNCCL's async error handling (the
    main thread may be blocked inside a device synchronisation that would never return)."""

    def __init__(self, poll_error, abort, timeout: float = 600.0, interval: float = 0.5, exit_code: int = 13,
                 on_fatal=None):
        self.poll_error, self.abort, self.timeout, self.interval = poll_error, abort, timeout, interval
        self.exit_code = exit_code
        self.on_fatal = on_fatal if on_fatal is not None else self._die
        self._pending = collections.deque()
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self.fired = None
        self._t = threading.Thread(target=self._run, name="imgcls-comm-watchdog", daemon=True)
        _WATCHDOGS.append(self)
        self._t.start()

    def arm(self, done) -> None:
        with self._lock:
            self._pending.append((time.monotonic(), done))

    def _die(self, msg: str) -> None:
        print(f"[imgcls] FATAL: {msg}; aborting the communicator and exiting ({self.exit_code})", file=sys.stderr,
              flush=True)
        os._exit(self.exit_code)

    def check_once(self) -> str | None:
        e = self.poll_error()
        if e:
            return f"RCCL communicator reported asynchronous error {e}"
        now = time.monotonic()
        with self._lock:
            while self._pending and self._pending[0][1].query():
                self._pending.popleft()
            if self._pending and now - self._pending[0][0] > self.timeout:
                return f"collectives enqueued {now - self._pending[0][0]:.0f} s ago have not completed (timeout " \
                       f"{self.timeout:.0f} s): a peer is dead or hung"
        return None

    def _run(self) -> None:
        while not self._stop.wait(self.interval):
            msg = self.check_once()
            if msg is not None and not self._stop.is_set():  # stopped meanwhile: an orderly teardown
                self.fired = msg
                try:
                    self.abort()
                finally:
                    self.on_fatal(msg)
                return

    def stop(self) -> None:
        self._stop.set()
        if self._t is not threading.current_thread():
            self._t.join(timeout=5)
        if self in _WATCHDOGS:
            _WATCHDOGS.remove(self)


def rccl_version() -> int:
    return _lib().rccl_version()
