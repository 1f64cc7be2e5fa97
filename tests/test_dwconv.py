"""Depthwise convolution kernels (csrc/dwconv.hip) against an fp32 PyTorch reference (F.conv2d with
groups=C on the same bf16-rounded operands): forward, data gradient, weight gradient, for the row-strip
kernels (K 3/5, stride 1/2) and the per-pixel kernels they replace, over odd sizes, widths below one
strip, asymmetric (TF "same") and symmetric padding with both parities of the left pad."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
CL = torch.channels_last

# (N, C, H, W, K, S, pt, pb, pl, pr)
CASES = [
    (2, 32, 17, 17, 3, 1, 1, 1, 1, 1),
    (2, 96, 28, 28, 3, 2, 0, 1, 0, 1),    # TF same, stride 2, even size
    (2, 24, 15, 13, 3, 2, 1, 1, 1, 1),    # odd sizes, pl odd
    (1, 144, 14, 14, 5, 1, 2, 2, 2, 2),
    (2, 40, 15, 15, 5, 2, 2, 2, 2, 2),    # odd size, TF same
    (2, 40, 16, 16, 5, 2, 1, 2, 1, 2),    # pl odd
    (1, 8, 7, 3, 5, 1, 2, 2, 2, 2),       # width below one strip
    (1, 16, 9, 5, 3, 2, 1, 1, 0, 1),      # narrow, pl even
    (3, 672, 7, 7, 5, 1, 2, 2, 2, 2),     # EfficientNet late stage (C > 256 chunk lanes... 84)
    (1, 2064, 5, 6, 3, 1, 1, 1, 1, 1),    # C/8 > 256: several channel passes per block in the weight gradient
]


def bf(t):
    return t.to(torch.bfloat16).float()


def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("rowstrip", [True, False])
@pytest.mark.parametrize("case", CASES)
def test_depthwise_fwd_dgrad_wgrad(case, rowstrip):
    from pytorch_imageclassification_distributed_amd.ops import hip
    C_ = hip.C
    n, c, h, w, k, s, pt, pb, pl, pr = case
    oh = (h + pt + pb - k) // s + 1
    ow = (w + pl + pr - k) // s + 1
    torch.manual_seed(hash(case) % 1000)
    x = bf(torch.randn(n, c, h, w, device=DEV))
    wt = bf(torch.randn(c, 1, k, k, device=DEV) * 0.2)
    dy = bf(torch.randn(n, c, oh, ow, device=DEV))
    xr = x.clone().requires_grad_(True)
    wr = wt.clone().requires_grad_(True)
    yr = F.conv2d(F.pad(xr, (pl, pr, pt, pb)), wr, None, s, 0, 1, c)
    assert yr.shape[2:] == (oh, ow)
    yr.backward(dy)

    xb = x.to(torch.bfloat16).contiguous(memory_format=CL)
    dyb = dy.to(torch.bfloat16).contiguous(memory_format=CL)
    wtt = wt.view(c, k * k).t().contiguous().to(torch.bfloat16)  # [taps][C]
    C_.dw_set_rowstrip(rowstrip)
    try:
        y = torch.empty(n, c, oh, ow, device=DEV, dtype=torch.bfloat16, memory_format=CL)
        C_.dw_fwd(xb, wtt, y, None, n, h, w, c, oh, ow, k, k, s, s, pt, pl)
        dx = torch.empty(n, c, h, w, device=DEV, dtype=torch.bfloat16, memory_format=CL)
        C_.dw_dgrad(dyb, wtt, dx, n, h, w, c, oh, ow, k, k, s, s, pt, pl)
        dw = torch.zeros(c, 1, k, k, device=DEV, dtype=torch.float32)
        C_.dw_wgrad(dyb, xb, dw, n, h, w, c, oh, ow, k, k, s, s, pt, pl)
        torch.cuda.synchronize()
    finally:
        C_.dw_set_rowstrip(True)
    assert rel(y, yr) < 1e-2, ("fwd", rel(y, yr))
    assert rel(dx, xr.grad) < 1e-2, ("dgrad", rel(dx, xr.grad))
    assert rel(dw, wr.grad) < 1e-4, ("wgrad", rel(dw, wr.grad))
