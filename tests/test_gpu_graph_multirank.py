"""Whole-step HIP-graph replay at N > 1: 2 ranks share one GPU, SyncBN over the one-shot peer
kernels (device-side call numbers, csrc/peer.hip), gradients summed over gloo after each replay.

Deterministic mode: the replayed run must leave every parameter and BN buffer bitwise equal to the eager run of
the same steps (same batches, same init), and the peer channels' device call counters must have advanced by the
calls of every replayed step.  Reference workload: the reference's default launch (Inception-v3, per-GPU batch
4, SyncBN, DDP; /root/reference/README.md:6, train.py:30,122,124,128) - Inception runs at its own 299 x 299 (the aux head needs Mixed_6e at 17 x 17); ResNet-18 at 64 x 64 keeps
the first case short (bench.py measures the replay speed).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, model, size):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), IMGCLS_PEER_TIMEOUT_S="60",
                      # fixed kernel choices in both processes (no per-process timing)
                      IMGCLS_CONV_STAGES="0", IMGCLS_WGRAD_BLOCKS="512", IMGCLS_WGRAD_STAGES="2",
                      IMGCLS_DIRECT_CONV="0")
    from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser
    from pytorch_imageclassification_distributed_amd.ops import hip
    from pytorch_imageclassification_distributed_amd.parallel import destroy, init_distributed, peer
    ctx = init_distributed(device="cuda", backend="gloo")
    hip.set_deterministic(True)
    dev = ctx.device
    g = torch.Generator(device="cpu").manual_seed(100 + rank)
    steps = 5
    xs = [torch.randn(4, 3, size, size, generator=g).to(dev) for _ in range(steps)]
    ys = [torch.randint(0, 7, (4,), generator=g).to(dev) for _ in range(steps)]

    def run(graph: bool):
        args = build_parser().parse_args([
            "--synthetic", "--model", model, "--image-size", str(size), "--batchsize", "4", "--num-classes", "7",
            "--num-workers", "0", "--lr", "1e-3", "--syncbn-comm", "peer",
            "--hip-graph", "on" if graph else "off"])
        torch.manual_seed(0)
        tr = Trainer(args, ctx)
        assert tr.syncbn_peer and tr.graph_capable()
        tr.net.train()
        losses = []
        for i in range(steps):
            losses.append(float(tr.reduce_loss(tr._epoch_step(xs[i], ys[i], i)).item()))
        torch.cuda.synchronize()
        assert (tr._graph is not None) == graph
        state = {k: v.detach().clone().cpu() for k, v in tr.model.state_dict().items()}
        return losses, state

    l_eager, s_eager = run(False)
    eager_chans = list(peer._CHANNELS.values())[-1]
    # eager: every call was launched by the host, so the device counter equals the host's count
    assert all(c.comm.device_seq() == c.comm.seq > 0 for c in eager_chans)
    l_graph, s_graph = run(True)
    assert peer.peer_errors() == 0
    # replays advance the device counters only (the host's count stops at the capture): 2 eager steps + the
    # capture recorded host calls, the device ran 5 steps' worth
    graph_chans = list(peer._CHANNELS.values())[-1]
    for ce, cg in zip(eager_chans, graph_chans):
        assert cg.comm.device_seq() == ce.comm.device_seq() > cg.comm.seq, (cg.comm.device_seq(), cg.comm.seq)
    assert l_eager == l_graph, (l_eager, l_graph)
    for k in s_eager:
        assert torch.equal(s_eager[k], s_graph[k]), k
    destroy()


@pytest.mark.parametrize("model,size", [("resnet18", 64), ("inceptionv3", 299)])
def test_graph_replay_two_ranks_bitwise_equals_eager(tmp_path, model, size):
    mp.spawn(_worker, args=(2, _port(), str(tmp_path), model, size), nprocs=2, join=True)
