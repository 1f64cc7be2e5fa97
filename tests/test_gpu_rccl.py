"""Native RCCL communicator (csrc/rccl_comm.cpp, parallel/rccl.py) on the GPU.

One GPU runs a world of one: rendezvous through the process group's TCPStore, ncclCommInitRank, in-place
collectives on the comm stream and their ordering against the compute stream, async-error polling, and the
gradient reducer with ``comm="rccl"`` (``force_collectives`` runs the bucket collectives in a world of
one).  Several ranks cannot share one GPU in an RCCL communicator, so the cross-GPU path is exercised by
the driver's multi-GPU runs (bench.py --comm-backend rccl)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ctx():
    from pytorch_imageclassification_distributed_amd.parallel import init_distributed
    return init_distributed(device="cuda")


def test_rccl_collectives_world_one():
    from pytorch_imageclassification_distributed_amd.parallel.rccl import RcclComm, rccl_version
    ctx = _ctx()
    assert rccl_version() > 0
    comm = RcclComm(None, ctx.device)
    try:
        for dt in (torch.float32, torch.bfloat16, torch.float64, torch.int64):
            x = (torch.arange(1 << 16, device=ctx.device) % 977).to(dt)
            ref = x.clone()
            # produced by a kernel on the compute stream right before: the collective must run after it
            y = x * 1
            comm.all_reduce_(y)
            comm.join()
            assert torch.equal(y, ref), dt
        for op in ("max", "min"):
            y = torch.randn(4096, device=ctx.device)
            ref = y.clone()
            comm.all_reduce_(y, op)
            comm.join()
            assert torch.equal(y, ref)
        b = torch.randn(1000, device=ctx.device)
        ref = b.clone()
        comm.broadcast_(b, 0)
        comm.join()
        assert torch.equal(b, ref)
        comm.check()
    finally:
        comm.close()
    with pytest.raises(RuntimeError):
        comm.C.rccl_all_reduce(comm.handle, torch.zeros(4, device=ctx.device), 0, 0)  # closed handle


@pytest.mark.parametrize("comm_dtype", [None, torch.bfloat16])
def test_reducer_native_rccl(comm_dtype):
    """GradReducer(comm="rccl"): bucket collectives on the native comm stream (world of one: a sum over one
    rank) leave the gradients as autograd produced them (bf16 transport: rounded to bf16)."""
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.parallel import GradReducer
    ctx = _ctx()
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(256, 512), nn.ReLU(), nn.Linear(512, 512), nn.ReLU(), nn.Linear(512, 10)).to(ctx.device)
    x = torch.randn(64, 256, device=ctx.device)
    model(x).square().mean().backward()
    ref = [p.grad.clone() for p in model.parameters()]
    for p in model.parameters():
        p.grad = None
    red = GradReducer(model, bucket_cap_mb=0.5, first_bucket_mb=0.25, comm_dtype=comm_dtype, comm="rccl",
                      force_collectives=True)
    try:
        assert red.rccl is not None and len(red.buckets) >= 2
        for _ in range(2):  # second step: after the bucket rebuild
            red.begin()
            model(x).square().mean().backward()
            scale = red.finish()
            assert scale == 1.0
            for p, r in zip(model.parameters(), ref):
                want = r.to(torch.bfloat16).float() if comm_dtype is not None else r
                torch.testing.assert_close(p.grad, want, rtol=1e-5, atol=1e-6)
    finally:
        red.rccl.close()
        red.remove_hooks()
