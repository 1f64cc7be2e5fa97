"""One-shot peer all-reduce (csrc/peer.hip, parallel/peer.py): ranks share one GPU, gloo carries the
handshake, the HIP kernel does the exchange through IPC-mapped buffers.

Checks exact fp64 sums against the sum computed from every rank's (seeded) input, over sizes that
cover one partial block up to the 32-block maximum, many back-to-back calls (both buffer parities,
sequence numbers far past the first), the side-stream asynchronous form, and a ResNet-50 SyncBN
training step whose statistics go through the peer kernel against the same step over gloo.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SIZES = [1, 7, 129, 511, 512, 513, 2049, 4097, 16384]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), IMGCLS_PEER_TIMEOUT_S="30")
    from pytorch_imageclassification_distributed_amd.parallel import init_distributed
    return init_distributed(device="cuda", backend="gloo")


def _inputs(n, world, it, dev):
    g = torch.Generator().manual_seed(1000 * n + it)
    xs = torch.randn(world, n, dtype=torch.float64, generator=g)
    return xs.to(dev)


def _unit_worker(rank, world, port):
    import torch.distributed as dist
    from pytorch_imageclassification_distributed_amd.parallel import peer
    ctx = _init(rank, world, port)
    dev = ctx.device
    assert peer.setup_peer_syncbn(dist.group.WORLD, dev, "peer")
    grp = dist.group.WORLD
    it = 0
    for rep in range(3):
        for n in SIZES:
            xs = _inputs(n, world, it, dev)
            want = xs[0].clone()
            for q in range(1, world):
                want += xs[q]  # rank order, as the kernel adds
            t = xs[rank].clone()
            if (it % 2) == 0:
                peer.stats_all_reduce_(t, grp)
            else:
                peer.stats_all_reduce_async(t, grp).wait()
            torch.cuda.synchronize()
            assert torch.equal(t, want), (rank, n, rep, (t - want).abs().max().item())
            it += 1
    # bursts with no host synchronisation in between (the stream runs far ahead of the host checks)
    outs = []
    for k in range(64):
        t = torch.full((300,), float(rank + 1 + k), dtype=torch.float64, device=dev)
        peer.stats_all_reduce_(t, grp)
        outs.append(t)
    torch.cuda.synchronize()
    for k, t in enumerate(outs):
        assert torch.all(t == sum(q + 1 + k for q in range(world))), k
    assert peer.peer_errors() == 0
    peer.teardown_peer_syncbn()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_peer_allreduce_exact(world):
    """Exact rank-ordered sums, both buffer parities (sync and side-stream calls alternate), 64-call bursts;
    world 8 is the driver's node size (8 processes sharing this one GPU: the flag / parity protocol and the
    bounded spin at the world size they will first meet)."""
    mp.spawn(_unit_worker, args=(world, _port()), nprocs=world, join=True)


def _model_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(IMGCLS_CONV_STAGES="0", IMGCLS_WGRAD_BLOCKS="512", IMGCLS_WGRAD_STAGES="2",
                      IMGCLS_DIRECT_CONV="0")
    from pytorch_imageclassification_distributed_amd.models import Classifier
    from pytorch_imageclassification_distributed_amd.ops import functional as Fx
    from pytorch_imageclassification_distributed_amd.ops import hip
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer, convert_sync_batchnorm, peer
    ctx = _init(rank, world, port)
    dev = ctx.device
    hip.set_deterministic(True)
    torch.manual_seed(0)
    x = torch.randn(8, 3, 64, 64, device=dev).to(torch.bfloat16).float()
    y = torch.randint(0, 7, (8,), device=dev)
    xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
    res = {}
    for mode in ("rccl", "peer"):  # rccl here = torch.distributed over gloo
        torch.manual_seed(1)
        m = Classifier("resnet50", 7).to(dev).to(memory_format=torch.channels_last)
        grp = dist.new_group(list(range(world)))
        convert_sync_batchnorm(m, grp)
        active = peer.setup_peer_syncbn(grp, dev, mode)
        assert active == (mode == "peer")
        red = GradReducer(m, bucket_cap_mb=4, first_bucket_mb=1)
        Fx.cross_entropy(m(xs), ys).backward()
        scale = red.finish()
        torch.cuda.synchronize()
        res[mode] = ({n: (p.grad * scale).float().cpu() for n, p in m.named_parameters()},
                     m.encoder.layer3[0].bn2.running_var.cpu())
    assert peer.peer_errors() == 0
    (ga, ra), (gb, rb) = res["rccl"], res["peer"]
    # same math, only the fp64 summation order of the statistics differs -> (nearly) identical
    assert torch.allclose(ra, rb, rtol=1e-5, atol=1e-7)
    for n in ga:
        cos = torch.nn.functional.cosine_similarity(ga[n].flatten(), gb[n].flatten(), dim=0).item()
        assert cos > 0.999, (n, cos)
    peer.teardown_peer_syncbn()
    dist.barrier()
    dist.destroy_process_group()


def test_peer_syncbn_resnet50_matches_torch_distributed(tmp_path):
    mp.spawn(_model_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)


def _timeout_worker(rank, world, port, out_dir):
    import time

    import torch.distributed as dist
    from pytorch_imageclassification_distributed_amd.parallel import peer
    ctx = _init(rank, world, port)
    os.environ["IMGCLS_PEER_TIMEOUT_S"] = "2"  # steady-state bound for this test: rank 1 arrives late
    dev = ctx.device
    grp = dist.group.WORLD
    assert peer.setup_peer_syncbn(grp, dev, "peer")
    t = torch.ones(64, dtype=torch.float64, device=dev)
    if rank == 1:
        time.sleep(6.0)  # past rank 0's 2 s bound: rank 0's call gives up, sets the error word
    peer.stats_all_reduce_(t, grp)
    torch.cuda.synchronize()
    raised = False
    try:
        peer.check_peer_errors("test")
    except peer.PeerTimeoutError:
        raised = True
    with open(os.path.join(out_dir, f"rank{rank}"), "w") as f:
        f.write("raised" if raised else "clean")
    peer.teardown_peer_syncbn()
    dist.barrier()
    dist.destroy_process_group()


def test_peer_timeout_is_fatal(tmp_path):
    """A peer that arrives after the spin bound (IMGCLS_PEER_TIMEOUT_S) makes the waiting rank's call give
    up with the device error word set; ``check_peer_errors`` (trainer: every log interval and epoch end)
    must turn that into an exception instead of letting training continue on wrong statistics."""
    mp.spawn(_timeout_worker, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    assert (tmp_path / "rank0").read_text() == "raised"
