"""Captured zero-initialised accumulations stay correct when eager launches run between HIP-graph replays.

The head's bias gradient (column sum with atomics), the split-K sgemm and the SE spatial reduce all start
from a zeroed output.  Trainer.fit replays a captured step, runs validation eagerly (which launches the same
ops on other buffers), then replays again: the first replay after validation must still zero its outputs.
ROCm 7's memset graph nodes did not (garbage bias gradients on the first replay of every epoch), so the
launchers zero with a kernel of their own (csrc/head.hip ``zero_f32_launch``).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _colsum_ref(x):
    return x.double().sum(0).float()


def test_colsum_and_sgemm_replay_after_eager_launches():
    from pytorch_imageclassification_distributed_amd.ops import hip
    C = hip.C
    dev = torch.device("cuda")
    torch.manual_seed(0)
    m, n, k = 64, 7, 4096
    x = torch.randn(m, n, device=dev)
    a = torch.randn(m, k, device=dev)  # 64 x 4096 @ 4096 x 64: few tiles, long K -> split-K into a zeroed output
    b = torch.randn(k, 64, device=dev)
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        db = torch.full((n,), 1e30, device=dev)  # garbage where the zeroing must land
        dx = torch.full((m, 64), 1e30, device=dev)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        C.colsum(x, None, db, m, n, n, False)
        hip._mm(a, b, dx, m, 64, k, k, 1, 64, 1)
    for rnd in range(4):
        db.fill_(1e30)
        dx.fill_(1e30)
        g.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(db, _colsum_ref(x), rtol=1e-5, atol=1e-4, msg=f"colsum replay {rnd}")
        torch.testing.assert_close(dx, a @ b, rtol=1e-3, atol=1e-2, msg=f"sgemm replay {rnd}")
        # eager launches of the same ops on other buffers between replays (validation does this)
        for _ in range(3):
            o = torch.empty(n * 3, device=dev)
            y = torch.randn(128, n * 3, device=dev)
            C.colsum(y, None, o, 128, n * 3, n * 3, False)
            big = torch.randn(256, 2048, device=dev)
            wb = torch.randn(64, 2048, device=dev)
            out = torch.empty(256, 64, device=dev)
            hip._mm(big, wb.t().contiguous(), out, 256, 64, 2048, 2048, 1, 64, 1)
        torch.cuda.synchronize()
