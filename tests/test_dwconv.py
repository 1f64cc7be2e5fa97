"""Depthwise convolution kernels (csrc/dwconv.hip) against an fp32 PyTorch reference (F.conv2d with
groups=C on the same bf16-rounded operands): forward, data gradient, weight gradient, for the row-strip
kernels (K 3/5, stride 1/2) and the per-pixel kernels they replace, over odd sizes, widths below one
strip, asymmetric (TF "same") and symmetric padding with both parities of the left pad."""
import copy

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


@pytest.mark.parametrize("rowstrip,wkr", [(True, 3), (True, 1), (False, 3)])
@pytest.mark.parametrize("case", CASES)
def test_depthwise_fwd_dgrad_wgrad(case, rowstrip, wkr):
    """Depthwise forward / data gradient / weight gradient against fp32 torch: row-strip kernels (5x5 weight
    gradient with 3 or 1 kernel rows per pass) and the per-pixel kernels."""
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
    C_.dw_set_wkr(wkr)
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
        C_.dw_set_wkr(3)
    assert rel(y, yr) < 1e-2, ("fwd", rel(y, yr))
    assert rel(dx, xr.grad) < 1e-2, ("dgrad", rel(dx, xr.grad))
    assert rel(dw, wr.grad) < 1e-4, ("wgrad", rel(dw, wr.grad))


@pytest.mark.parametrize("k,s,hw,c", [(3, 1, 14, 96), (5, 2, 15, 40), (3, 2, 16, 144), (5, 1, 7, 672)])
def test_depthwise_fused_bn_backward(k, s, hw, c):
    """1x1 conv -> BN -> SiLU -> depthwise (exclusive consumer) -> BN -> SiLU: the depthwise data-gradient
    kernel emits dz and the first BN's backward partial sums (BwdLink); gradients match fp32 autograd and
    the unfused path."""
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.ops import hip
    from pytorch_imageclassification_distributed_amd.ops.functional import conv_padding
    torch.manual_seed(k * 100 + c)
    cin = 32
    pw = nn.Conv2d(cin, c, 1, bias=False).to(DEV).to(memory_format=CL)
    bn0 = nn.BatchNorm2d(c, eps=1e-3).to(DEV)
    dw = nn.Conv2d(c, c, k, s, 0, groups=c, bias=False).to(DEV).to(memory_format=CL)
    dw.tf_same = True
    bn1 = nn.BatchNorm2d(c, eps=1e-3).to(DEV)
    with torch.no_grad():
        pw.weight.copy_(bf(pw.weight))
        dw.weight.copy_(bf(dw.weight))
        bn0.weight.uniform_(0.5, 1.5)
        bn0.bias.uniform_(-0.5, 0.5)
    x = bf(torch.randn(4, cin, hw, hw, device=DEV))
    g = None
    grads = {}
    keep = hip.DW_LINK
    hip.DW_LINK = True  # opt-in in the trainer (measured slower on EfficientNet-B0); tested here
    for fused in (True, False):
        for m in (pw, bn0, dw, bn1):
            for p_ in m.parameters():
                p_.grad = None
        xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
        before = hip.FUSED_BWD_COUNT[0]
        a = hip.conv_bn_act(xb, pw, bn0, "silu", None)
        out = hip.conv_bn_act(a, dw, bn1, "silu", None, exclusive_input=fused)
        if g is None:
            g = bf(torch.randn(out.shape, device=DEV))
        out.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
        torch.cuda.synchronize()
        assert (hip.FUSED_BWD_COUNT[0] > before) == fused
        grads[fused] = [xb.grad.float()] + [p_.grad.float().clone() for m in (pw, bn0, dw, bn1) for p_ in m.parameters()]
    hip.DW_LINK = keep
    # fp32 reference
    xr = x.clone().requires_grad_(True)
    ps = [p_.detach().clone().requires_grad_(True) for m in (pw, bn0, dw, bn1) for p_ in m.parameters()]
    pt, pb, pl, pr = conv_padding(dw, hw, hw)
    z0 = F.conv2d(xr, ps[0])
    a0 = F.silu(F.batch_norm(z0, None, None, ps[1], ps[2], training=True, eps=1e-3))
    z1 = F.conv2d(F.pad(a0, (pl, pr, pt, pb)), ps[3], None, s, 0, 1, c)
    ref = F.silu(F.batch_norm(z1, None, None, ps[4], ps[5], training=True, eps=1e-3))
    ref.backward(g)
    refs = [xr.grad] + [p_.grad for p_ in ps]
    for i, r in enumerate(refs):
        assert rel(grads[True][i], r) < 3e-2, (i, rel(grads[True][i], r))
        assert rel(grads[True][i], grads[False][i]) < 3e-2, (i, rel(grads[True][i], grads[False][i]))


@pytest.mark.parametrize("k,s,hw,c", [(3, 1, 14, 96), (5, 2, 15, 40), (3, 2, 16, 144), (5, 1, 7, 672)])
def test_depthwise_forward_bn_statistics(k, s, hw, c):
    """depthwise -> BN (train) -> SiLU with the BN's batch statistics produced by the depthwise forward
    (ops/_hip/convbn.py DW_STATS, csrc/dwconv.hip EPI 2) against the BN's own statistics pass and fp32 torch:
    output, running mean / var (about a non-zero pivot, with a large channel mean), and the backward."""
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.ops import hip
    from pytorch_imageclassification_distributed_amd.ops.functional import conv_padding
    torch.manual_seed(k * 10 + c)
    dw = nn.Conv2d(c, c, k, s, 0, groups=c, bias=False).to(DEV).to(memory_format=CL)
    dw.tf_same = True
    bn = nn.BatchNorm2d(c, eps=1e-3).to(DEV)
    with torch.no_grad():
        dw.weight.copy_(bf(dw.weight.abs() + 0.05))  # positive taps: channel means of ~10 std from the +3 input
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.2, 0.2)  # the statistics pivot
    x = bf(torch.randn(4, c, hw, hw, device=DEV) + 3.0)
    g = bf(torch.randn(4, c, (hw + s - 1) // s, (hw + s - 1) // s, device=DEV))
    res = {}
    keep = hip.DW_STATS
    keep_px = hip.C.dw_set_stats_min_px(0)  # fuse every geometry here (the trainer gates on pixels per block)
    try:
        for fused in (True, False):
            hip.DW_STATS = fused
            b = copy.deepcopy(bn)
            xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
            before = hip.DW_STATS_COUNT[0]
            out = hip.conv_bn_act(xb, dw, b, "silu", None)
            assert (hip.DW_STATS_COUNT[0] > before) == fused
            out.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
            torch.cuda.synchronize()
            res[fused] = (out.float(), b.running_mean.clone(), b.running_var.clone(), xb.grad.float(),
                          [p_.grad.float().clone() for p_ in b.parameters()])
            dw.weight.grad = None
    finally:
        hip.DW_STATS = keep
        hip.C.dw_set_stats_min_px(keep_px)
    br = copy.deepcopy(bn)
    xr = x.clone().requires_grad_(True)
    pt, pb, pl, pr = conv_padding(dw, hw, hw)
    z = F.conv2d(F.pad(xr, (pl, pr, pt, pb)), dw.weight.detach(), None, s, 0, 1, c)
    z = z + (bf(z) - z).detach()  # the stored output is bf16
    ref = F.silu(br(z))
    ref.backward(g)
    for fused in (True, False):
        o, rm, rv, gx, gp = res[fused]
        assert rel(o, ref) < 2e-2, (fused, rel(o, ref))
        assert torch.allclose(rm, br.running_mean, rtol=1e-3, atol=1e-3), fused
        assert torch.allclose(rv, br.running_var, rtol=1e-2, atol=1e-3), fused
        assert rel(gx, xr.grad) < 3e-2, (fused, rel(gx, xr.grad))
        for a, r in zip(gp, br.parameters()):
            assert rel(a, r.grad) < 3e-2, fused
    assert rel(res[True][0], res[False][0]) < 1e-2
