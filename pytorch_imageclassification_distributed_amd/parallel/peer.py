"""One-shot peer all-reduce for the SyncBN statistics.

The reference's SyncBatchNorm runs two small blocking collectives per BN layer and step
(reference train.py:124 -> torch/nn/modules/_functions.py:74 and :159).  They are latency-bound:
<= 33 KB each, 2 x 53 per ResNet-50 step.  On one node every GPU reaches every other one over its
own xGMI link, so instead of a ring (2(W-1) dependent hops) each rank pushes its payload straight
into every peer's IPC-mapped buffer and sums what the peers pushed into its own - one kernel,
one hop (``csrc/peer.hip``).

``PeerAllReduce`` is one channel: a buffer per rank, the peers' buffers mapped here, and a call
sequence number.  Calls on one channel must be issued in the same order on every rank and on one
stream; SyncBN uses two channels - the forward statistics on the compute stream and the backward
sums on a side stream (overlapping the consuming conv's weight gradient).

Creation is collective over the group (handles are exchanged with ``all_gather_object``), ends
with a self-check (three calls against the exact expected sums, both buffer parities), and any
failure falls back to ``torch.distributed`` (RCCL) with a warning, never to a wrong answer.  Once
training runs, a call that timed out waiting for a peer (``IMGCLS_PEER_TIMEOUT_S``, default 120 s)
leaves a device error word set: ``check_peer_errors`` (called by the trainer at every log interval
and epoch end, and by the bench) turns it into an exception, so a run whose statistics may have
summed stale slots stops instead of training on.
"""
from __future__ import annotations

import os
import socket
import warnings

import torch
import torch.distributed as dist

_CHANNELS: dict = {}  # id(group) -> (fwd channel, bwd channel)


def _agree(ok: bool, group, device) -> bool:
    """True only if ``ok`` holds on every rank of the group (collective)."""
    flag = torch.tensor([0 if ok else 1], dtype=torch.int32)
    if dist.get_backend(group) == "nccl":
        flag = flag.to(device)
    dist.all_reduce(flag, group=group)
    return int(flag.item()) == 0


class PeerAllReduce:
    """One channel.  Construction is collective and never leaves the group mid-handshake: each
    step's success is agreed on by all ranks before the next step (a rank that failed to map a
    peer's buffer must not let the others start kernels that would wait for it)."""

    def __init__(self, group, device: torch.device, timeout_s: float = 120.0):
        from .. import _ext
        self.timeout_s = timeout_s
        C = _ext.load()
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device
        self.max_elems = int(C.PEER_MAX_ELEMS)
        self.comm = None
        handle, why = None, ""
        with torch.cuda.device(device):
            try:
                self.comm = C.PeerComm(self.rank, self.world, float(timeout_s))
                torch.cuda.synchronize(device)
                handle = bytes(self.comm.handle())
            except Exception as e:  # noqa: BLE001
                why = f"rank {self.rank}: buffer / IPC handle: {e}"
            handles = [None] * self.world
            dist.all_gather_object(handles, handle, group=group)
            ok = all(h is not None for h in handles)
            if ok:
                try:
                    self.comm.open(handles)
                    torch.cuda.synchronize(device)
                except Exception as e:  # noqa: BLE001
                    ok, why = False, f"rank {self.rank}: hipIpcOpenMemHandle: {e}"
            if not _agree(ok, group, device):
                self.close()
                raise RuntimeError(why or "a peer could not export or map its buffer")

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over the group on the current stream (fp64, contiguous)."""
        self.comm.all_reduce_(t, t)
        return t

    def error(self) -> int:
        """Non-zero once any call timed out waiting for a peer (reads a device word: syncs)."""
        return int(self.comm.error())

    def self_check(self, timeout_s: float = 15.0, steady_timeout_s: float = 120.0) -> bool:
        """Three calls (both buffer parities, then a re-use) against the exact sums (collective).
        The calls wait at most ``timeout_s`` for the peers (a transport whose stores never arrive
        costs seconds, not 3 x the steady-state bound); later calls get ``steady_timeout_s``."""
        n = min(5000, self.max_elems)
        ok = True
        try:
            base = torch.arange(1, n + 1, dtype=torch.float64, device=self.device)
            want = base * (self.world * (self.world + 1) / 2)
            self.comm.set_timeout(float(timeout_s))
            try:
                for k in range(3):
                    t = base * (self.rank + 1) + k
                    self.all_reduce_(t)
                    ok &= bool(torch.equal(t, want + k * self.world))  # syncs: a timed-out call ends the check
                    if not ok:
                        break
                torch.cuda.synchronize(self.device)
                return ok and self.error() == 0
            finally:
                self.comm.set_timeout(float(steady_timeout_s))
        except Exception as e:  # noqa: BLE001 - a launch / HIP error on this rank is a failed check, so
            # every rank still reaches the collective agreement that follows (no mismatched collectives)
            warnings.warn(f"SyncBN peer self-check raised on rank {self.rank}: {e}")
            return False

    def close(self) -> None:
        if self.comm is not None:
            self.comm.close()
            self.comm = None


class PeerWork:
    """``dist.Work``-like handle: ``wait()`` orders the current stream after the side-stream call."""

    def __init__(self, ev: torch.cuda.Event):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)
        return True


_SIDE: dict = {}


def _side_stream(dev):
    s = _SIDE.get(dev)
    if s is None:
        lo, hi = torch.cuda.Stream.priority_range()
        s = _SIDE[dev] = torch.cuda.Stream(device=dev, priority=hi)
    return s


def _same_host(group) -> bool:
    names = [None] * dist.get_world_size(group)
    dist.all_gather_object(names, socket.gethostname(), group=group)
    return len(set(names)) == 1


def setup_peer_syncbn(group, device: torch.device, mode: str = "auto") -> bool:
    """Create the SyncBN peer channels for ``group`` (collective).  mode: auto | peer | rccl.

    auto = peer when every rank of the group is on this host and the self-check passes; peer =
    the same but a failure raises.  Returns whether the peer path is active."""
    mode = os.environ.get("IMGCLS_SYNCBN_COMM", mode)
    if group is None or mode == "rccl" or device.type != "cuda" or dist.get_world_size(group) == 1:
        return False
    world = dist.get_world_size(group)
    tmo = float(os.environ.get("IMGCLS_PEER_TIMEOUT_S", "120"))
    chans = []
    try:
        from .. import _ext
        if world > int(_ext.load().PEER_MAX_WORLD):  # same answer on every rank
            raise RuntimeError(f"world {world} above the peer kernel's limit")
        if not _same_host(group):
            raise RuntimeError("ranks span several hosts")
        for _ in range(2):  # forward (compute stream) and backward (side stream) channels
            chans.append(PeerAllReduce(group, device, tmo))
        check_s = float(os.environ.get("IMGCLS_PEER_CHECK_TIMEOUT_S", "15"))
        ok, err = True, None
        for c in chans:
            try:  # a local exception (launch error, ...) is a failed check: this rank still reaches _agree
                ok = c.self_check(check_s, tmo) and ok
            except Exception as e:  # noqa: BLE001
                ok, err = False, e
        if not _agree(ok, group, device):  # every rank must agree, or ranks would mix transports
            if err is not None:
                raise RuntimeError(f"self-check raised on this rank: {err}") from err
            raise RuntimeError("self-check failed on some rank")
    except Exception as e:  # noqa: BLE001 - any failure means the torch.distributed path
        for c in chans:  # channels already mapped (a failure in the second one leaks none)
            c.close()
        if mode == "peer":
            raise
        warnings.warn(f"SyncBN peer all-reduce disabled, using torch.distributed: {e}")
        return False
    _CHANNELS[id(group)] = tuple(chans)
    return True


def teardown_peer_syncbn() -> None:
    for chans in _CHANNELS.values():
        for c in chans:
            c.close()
    _CHANNELS.clear()


def peer_active(group) -> bool:
    return group is not None and id(group) in _CHANNELS


def peer_errors() -> int:
    """Sum of the device error words of every channel (timeouts); syncs."""
    return sum(c.error() for chans in _CHANNELS.values() for c in chans)


class PeerTimeoutError(RuntimeError):
    """A SyncBN peer exchange gave up waiting for a peer: its statistics may be wrong."""


def check_peer_errors(where: str = "") -> None:
    """Raise ``PeerTimeoutError`` if any peer call timed out (syncs the device; call it at log
    intervals, not per step).  The run must stop: the timed-out rank summed whatever the slots held and
    its call sequence no longer matches its peers'."""
    if not _CHANNELS:
        return
    n = peer_errors()
    if n:
        raise PeerTimeoutError(f"SyncBN peer all-reduce timed out waiting for a peer{' (' + where + ')' if where else ''}"
                               f": {n} channel error word(s) set; the statistics of that step are invalid")


class SyncBNMismatchError(RuntimeError):
    pass


def check_syncbn_consistency(module, group=None, where: str = "") -> None:
    """Steady-state guard for SyncBN (collective; call every ``--syncbn-check-every`` steps and at epoch end):
    every rank must hold bitwise the same BN running statistics, because each rank sums the same per-rank
    payloads in rank order (peer path) or receives the same all-reduce result (RCCL).  A transport fault - a
    stale or torn slot - shows up here as a mismatch, and the run stops instead of training on diverged
    statistics.  One flat pass: the running buffers are concatenated once and reduced to a position-weighted
    checksum pair (a swapped or shifted buffer changes it too), then one 6-value all-reduce.  Non-finite
    running statistics on every rank (a diverged run) are reported as divergence; on some ranks only, as the
    transport mismatch they are."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    bufs = [b for n, b in module.named_buffers() if "running_" in n]
    if not bufs:
        return
    flat = torch.cat([b.detach().reshape(-1) for b in bufs]).double()
    w = torch.arange(1, flat.numel() + 1, dtype=torch.float64, device=flat.device)
    s = torch.stack([flat.sum(), (flat * w).sum()])
    fin = torch.isfinite(s).all()
    s = torch.where(fin, s, torch.zeros_like(s))
    nf = (~fin).double().reshape(1)
    both = torch.cat([s, -s, nf, -nf])  # MAX of x and of -x: the max and the min over ranks in one reduce
    dist.all_reduce(both, op=dist.ReduceOp.MAX, group=group)
    any_nf, all_nf = both[4].item() > 0, -both[5].item() > 0
    if all_nf:
        raise SyncBNMismatchError(f"SyncBN running statistics are not finite on every rank{' (' + where + ')' if where else ''}"
                                  ": the run diverged (not a transport fault)")
    if any_nf:  # identical inputs on every rank cannot leave only some of them non-finite: a stale / torn slot
        raise SyncBNMismatchError(f"SyncBN running statistics are not finite on some ranks only{' (' + where + ')' if where else ''}"
                                  ": the ranks' statistics differ (transport fault)")
    if not torch.equal(both[:2], -both[2:4]):
        raise SyncBNMismatchError(f"SyncBN running statistics differ between ranks{' (' + where + ')' if where else ''}:"
                                  f" checksum max {both[:2].tolist()} vs min {(-both[2:4]).tolist()}")


def peer_channel(group, which: int):
    """The group's forward (0, compute stream) or backward (1, side stream) channel, or None."""
    chans = _CHANNELS.get(id(group)) if group is not None else None
    return chans[which] if chans is not None else None


def side_stream(dev):
    """High-priority stream of the backward channel (created on first use)."""
    return _side_stream(dev)


def stats_all_reduce_(t: torch.Tensor, group) -> None:
    """Blocking-in-stream-order sum of a SyncBN statistics vector (forward / backward)."""
    chans = _CHANNELS.get(id(group))
    if chans is None or t.numel() > chans[0].max_elems:
        dist.all_reduce(t, group=group)
        return
    chans[0].all_reduce_(t)


def stats_all_reduce_async(t: torch.Tensor, group):
    """Sum on a side stream; returns a handle whose ``wait()`` orders the current stream after it."""
    chans = _CHANNELS.get(id(group))
    if chans is None or t.numel() > chans[1].max_elems:
        return dist.all_reduce(t, group=group, async_op=True)
    cur = torch.cuda.current_stream(t.device)
    side = _side_stream(t.device)
    side.wait_stream(cur)
    with torch.cuda.stream(side):
        chans[1].all_reduce_(t)
        ev = torch.cuda.Event()
        ev.record(side)
    t.record_stream(side)
    return PeerWork(ev)
