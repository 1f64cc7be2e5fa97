"""Multi-process (gloo, world_size 2) tests of the parallel layer - no cluster needed.

* object all_gather / reduce_tensor (reference ddp_utils.py)
* GradReducer: W=2 half batches == W=1 full batch gradients (DDP equivalence),
  with SyncBN (cross-replica statistics) so BN layers see the global batch
* SyncBN forward/backward == single-process BN on the concatenated batch
* parameter broadcast at construction (DDP's _sync_module_states)
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _setup(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from pytorch_imageclassification_distributed_amd.parallel import init_distributed
    return init_distributed(device="cpu", backend="gloo")


def _run(fn, world=2):
    port = _port()
    mp.spawn(fn, args=(world, port), nprocs=world, join=True)


# ---------------------------------------------------------------------------
def _w_comm(rank, world, port):
    ctx = _setup(rank, world, port)
    import ddp_utils
    out = ddp_utils.all_gather({"rank": rank, "pad": "x" * (10 + 50 * rank)})
    assert [o["rank"] for o in out] == [0, 1] and len(out[1]["pad"]) == 60
    t = ddp_utils.reduce_tensor(torch.tensor([float(rank + 1)]))
    assert t.item() == pytest.approx(1.5)
    from pytorch_imageclassification_distributed_amd.parallel import all_gather_tensor
    g = all_gather_tensor(torch.tensor([rank, 10 + rank]))
    assert g.tolist() == [[0, 10], [1, 11]]
    assert ctx.world_size == 2


def test_object_all_gather_and_reduce():
    _run(_w_comm)


# ---------------------------------------------------------------------------
def _model(seed):
    from pytorch_imageclassification_distributed_amd.models import Classifier
    torch.manual_seed(seed)
    return Classifier("resnet18", 4)


def _w_ddp(rank, world, port):
    _setup(rank, world, port)
    import torch.nn.functional as F
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer, convert_sync_batchnorm
    torch.manual_seed(123)
    x = torch.randn(8, 3, 16, 16)
    y = torch.randint(0, 4, (8,))
    # reference: one process, full batch, plain BN
    ref = _model(0)
    F.cross_entropy(ref(x), y).backward()
    # distributed: different init on rank 1 (must be overwritten by the broadcast)
    m = _model(rank)
    convert_sync_batchnorm(m)
    red = GradReducer(m, bucket_cap_mb=0.5, first_bucket_mb=0.1)
    assert len(red.buckets) > 2
    for it in range(2):  # second iteration runs on the rebuilt bucket layout
        for p in m.parameters():
            p.grad = None
        xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
        F.cross_entropy(m(xs), ys).backward()
        scale = red.finish()
    for (n, p), (_n, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p.grad * scale, q.grad, rtol=1e-4, atol=1e-5), n


def test_grad_reducer_matches_single_process():
    _run(_w_ddp)


# ---------------------------------------------------------------------------
def _w_syncbn(rank, world, port):
    _setup(rank, world, port)
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.parallel import sync_batch_norm
    import torch.distributed as dist
    torch.manual_seed(7)
    x = torch.randn(6, 5, 4, 4) * 3 + 1
    gy = torch.randn(6, 5, 4, 4)
    bn_ref = nn.BatchNorm2d(5)
    xr = x.clone().requires_grad_(True)
    yr = bn_ref(xr)
    yr.backward(gy)
    bn = nn.BatchNorm2d(5)
    sl = slice(0, 2) if rank == 0 else slice(2, 6)  # unequal per-rank counts
    xs = x[sl].clone().requires_grad_(True)
    ys = sync_batch_norm(xs, bn, dist.group.WORLD)
    assert torch.allclose(ys, yr[sl], atol=1e-5)
    ys.backward(gy[sl])
    assert torch.allclose(xs.grad, xr.grad[sl], atol=1e-5)
    assert torch.allclose(bn.running_mean, bn_ref.running_mean, atol=1e-6)
    assert torch.allclose(bn.running_var, bn_ref.running_var, atol=1e-5)
    gw = bn.weight.grad.clone()
    dist.all_reduce(gw)
    assert torch.allclose(gw, bn_ref.weight.grad, atol=1e-4)


def test_syncbn_matches_global_batch_norm():
    _run(_w_syncbn)


# ---------------------------------------------------------------------------
def _w_train(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import train
    ck = os.environ["_TEST_CKPT"]
    hist = train.main(["--synthetic", "--model", "resnet18", "--image-size", "16", "--device", "cpu",
                       "--batchsize", "8", "--epochs", "2", "--num-workers", "0", "--synthetic-train-size", "64",
                       "--synthetic-val-size", "16", "--ckpt-dir", ck, "--lr", "1e-3", "--no-progress",
                       "--val-batchsize", "4", "--resume", "none"])
    assert len(hist) == 2
    import json
    with open(os.path.join(ck, f"hist{rank}.json"), "w") as f:
        json.dump(hist, f)


def test_train_cli_two_processes(tmp_path):
    os.environ["_TEST_CKPT"] = str(tmp_path)
    _run(_w_train)
    import json
    h0 = json.load(open(tmp_path / "hist0.json"))
    h1 = json.load(open(tmp_path / "hist1.json"))
    assert [r["val_acc"] for r in h0] == [r["val_acc"] for r in h1]  # combined accuracy on all ranks
    assert [r["train_loss"] for r in h0] == pytest.approx([r["train_loss"] for r in h1])  # globally averaged loss
    assert (tmp_path / "resnet18" / "best_model").exists()


# ---------------------------------------------------------------------------
def _w_fault(rank, world, port, marker, timeout_min):
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from pytorch_imageclassification_distributed_amd.parallel import init_distributed
    init_distributed(device="cpu", backend="gloo", timeout_min=timeout_min)
    dist.barrier()
    if rank == 1:
        os._exit(17)  # injected fault: the rank disappears without a clean shutdown
    t0 = time.time()
    try:
        for _ in range(1000):
            dist.all_reduce(torch.ones(1024))
            time.sleep(0.01)
        outcome = "no-error"
    except Exception as e:  # noqa: BLE001 - any collective error is the expected outcome
        outcome = type(e).__name__
    with open(marker, "w") as f:
        f.write(f"{outcome} {time.time() - t0:.2f}")
    os._exit(0)


def test_rank_failure_is_detected(tmp_path):
    """Fault injection: when a peer dies mid-run the surviving rank's collective fails
    within the process-group timeout instead of hanging."""
    ctxm = mp.get_context("spawn")
    port, marker = _port(), str(tmp_path / "rank0.txt")
    procs = [ctxm.Process(target=_w_fault, args=(r, 2, port, marker, 0.5)) for r in range(2)]
    for p_ in procs:
        p_.start()
    for p_ in procs:
        p_.join(timeout=120)
    alive = [p_ for p_ in procs if p_.is_alive()]
    for p_ in alive:
        p_.kill()
    assert not alive, "a rank hung after its peer died"
    outcome, secs = open(marker).read().split()
    assert outcome != "no-error"
    assert float(secs) < 60


def _w_buffers(rank, world, port):
    _setup(rank, world, port)
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer
    m = nn.Sequential(nn.Conv2d(3, 4, 1), nn.BatchNorm2d(4))
    torch.manual_seed(0)
    for p_ in m.parameters():
        nn.init.normal_(p_)
    red = GradReducer(m, broadcast=False)
    m[1].running_mean.fill_(float(rank + 1))
    m[1].num_batches_tracked.fill_(rank + 5)
    red.sync_buffers()
    assert torch.all(m[1].running_mean == 1.0) and int(m[1].num_batches_tracked) == 5


def test_broadcast_buffers():
    """DDP broadcast_buffers parity (X3): rank 0's BN buffers overwrite the other ranks'."""
    _run(_w_buffers)


# ---------------------------------------------------------------------------
def _w_shapes(rank, world, port):
    _setup(rank, world, port)
    from pytorch_imageclassification_distributed_amd.models import Classifier
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer
    m = Classifier("resnet18", 4 if rank == 0 else 5)  # head differs on rank 1
    with pytest.raises(RuntimeError, match="parameter list differs"):
        GradReducer(m)


def test_grad_reducer_verifies_param_shapes():
    """X1: DDP's _verify_param_shape_across_processes - mismatched models fail loudly at construction."""
    _run(_w_shapes)


def _w_order(rank, world, port):
    _setup(rank, world, port)
    import torch.nn.functional as F
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer
    m = _model(0)
    red = GradReducer(m, bucket_cap_mb=0.5, first_bucket_mb=0.1)
    x, y = torch.randn(4, 3, 16, 16), torch.randint(0, 4, (4,))
    F.cross_entropy(m(x), y).backward()
    if rank == 1:  # pretend this rank saw a different gradient-ready order
        red._ready_order = list(reversed(red._ready_order))
    red.finish()
    import torch.distributed as dist
    layouts = [None] * world
    dist.all_gather_object(layouts, [(s, e, list(i)) for s, e, i in red.buckets])
    assert layouts[0] == layouts[1]  # rank 0's observed order is the one every rank rebuilt with
    dist.barrier()
    dist.destroy_process_group()  # clean gloo teardown before exit (an exit with live gloo threads can abort)


def test_bucket_rebuild_uses_rank0_order():
    _run(_w_order)


def _w_overlap(rank, world, port):
    _setup(rank, world, port)
    import torch.distributed as dist
    import torch.nn.functional as F
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer
    m = _model(0)
    red = GradReducer(m, bucket_cap_mb=0.5, first_bucket_mb=0.1)
    seen = []  # gradients already arrived when each bucket's collective was issued
    orig = red._launch

    def spy(b):
        seen.append(sum(red.got))
        orig(b)
    red._launch = spy
    x, y = torch.randn(4, 3, 16, 16), torch.randint(0, 4, (4,))
    for _ in range(2):  # first step records the ready order, second runs on the rebuilt buckets
        seen.clear()
        red.begin()
        F.cross_entropy(m(x), y).backward()
        nb, launched = len(red.buckets), sum(red.launched)
        assert nb > 2
        # every bucket's all-reduce is already issued when backward returns (nothing waits for finish())
        assert launched == nb, (launched, nb)
        # and the first one went out while most gradients were still being computed
        assert seen[0] < len(red.params) // 2, (seen[:3], len(red.params))
        red.finish()
    dist.barrier()
    dist.destroy_process_group()


def test_bucket_collectives_issued_during_backward():
    """the bucket all-reduces are in flight before backward ends (DDP-style overlap), not
    issued from finish()."""
    _run(_w_overlap)


def _w_syncbn_guard(rank, world, port):
    _setup(rank, world, port)
    import torch.distributed as dist
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.parallel import SyncBNMismatchError, check_syncbn_consistency
    torch.manual_seed(0)
    m = nn.Sequential(nn.Conv2d(3, 8, 3), nn.BatchNorm2d(8), nn.ReLU(), nn.Conv2d(8, 8, 1), nn.BatchNorm2d(8))
    check_syncbn_consistency(m, None, "identical")  # same buffers on both ranks: passes
    if rank == 1:
        with torch.no_grad():
            m[4].running_var[3] += 1e-6  # one element on one rank
    with pytest.raises(SyncBNMismatchError, match="differ between ranks"):
        check_syncbn_consistency(m, None, "perturbed")
    dist.barrier()
    dist.destroy_process_group()


def test_syncbn_consistency_guard():
    """Steady-state SyncBN guard: diverged running statistics on any rank stop the run on
    every rank (the check is collective, so all ranks raise together)."""
    _run(_w_syncbn_guard)
