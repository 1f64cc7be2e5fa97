"""Residual blocks on the HIP path: gradients with the fused paired-gradient slots must equal the
gradients autograd produces when the two contributions are summed separately."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


class _SameState:
    """Restores a module's buffers (BN running statistics, batch counters) before every run.  Train-mode
    passes update the running mean, and the HIP BN kernels sum their statistics about it (the shifted-data
    pivot), so two passes compared against each other must start from the same buffers - otherwise they
    differ by the pivot's rounding, which random-init BatchNorm stacks amplify."""

    def __init__(self, module):
        self.m = module
        self.saved = [b.detach().clone() for b in module.buffers()]

    def __call__(self):
        with torch.no_grad():
            for b, s in zip(self.m.buffers(), self.saved):
                b.copy_(s)


def _grads(block, x, use_slots):
    """use_slots=False: no paired slots and no BN-backward fusion (plain autograd accumulation +
    standalone BN reduce kernel) - the reference the fused path must match."""
    from pytorch_imageclassification_distributed_amd.ops import functional as Fx
    from pytorch_imageclassification_distributed_amd.ops import hip
    orig, orig_fuse = Fx.grad_slot, hip.FUSE_BN_BWD
    block._imgcls_same_state = getattr(block, "_imgcls_same_state", None) or _SameState(block)
    block._imgcls_same_state()
    if not use_slots:
        Fx.grad_slot = lambda t, n=2: None
        hip.FUSE_BN_BWD = False
    try:
        for p in block.parameters():
            p.grad = None
        xx = x.clone().requires_grad_(True)
        out = block(xx)
        (out.float() * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum().backward()
    finally:
        Fx.grad_slot = orig
        hip.FUSE_BN_BWD = orig_fuse
    return xx.grad.float(), {n: p.grad.float().clone() for n, p in block.named_parameters()}


@pytest.mark.parametrize("kind", ["basic_id", "basic_ds", "bottle_id", "bottle_ds", "chain"])
def test_block_slots(kind):
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.models.resnet import BasicBlock, Bottleneck, _conv1x1
    torch.manual_seed(0)
    if kind == "basic_id":
        blk, cin = BasicBlock(64, 64), 64
    elif kind == "basic_ds":
        blk, cin = BasicBlock(64, 128, 2, nn.Sequential(_conv1x1(64, 128, 2), nn.BatchNorm2d(128))), 64
    elif kind == "bottle_id":
        blk, cin = Bottleneck(256, 64), 256
    elif kind == "bottle_ds":
        blk, cin = Bottleneck(256, 128, 2, nn.Sequential(_conv1x1(256, 512, 2), nn.BatchNorm2d(512))), 256
    else:  # two blocks: the second block's fused dgrad runs the first block's BN3 backward reduce
        blk = nn.Sequential(Bottleneck(256, 128, 2, nn.Sequential(_conv1x1(256, 512, 2), nn.BatchNorm2d(512))),
                            Bottleneck(512, 128))
        cin = 256
    blk = blk.to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(4, cin, 16, 16, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    from pytorch_imageclassification_distributed_amd.ops import hip
    gx0, gp0 = _grads(blk, x, False)
    before = hip.FUSED_BWD_COUNT[0]
    gx1, gp1 = _grads(blk, x, True)
    fused = hip.FUSED_BWD_COUNT[0] - before
    # chain: + the first block's deferred downsample BN, whose partial sums ride in the same epilogue as its BN3's
    chain = 6 if (hip.RES_DEFER and hip.DS_FUSE and hip.RELU_MASK) else 5
    expect = {"basic_id": 1, "basic_ds": 1, "bottle_id": 2, "bottle_ds": 2, "chain": chain}[kind]
    assert fused == expect, (kind, fused)
    err = lambda a, b: ((a - b).abs().max() / b.abs().max().clamp(min=1e-6)).item()  # noqa: E731
    assert err(gx1, gx0) < 2e-2, err(gx1, gx0)
    for n in gp0:
        assert err(gp1[n], gp0[n]) < 2e-2, (n, err(gp1[n], gp0[n]))


def _cos(a, b):
    a, b = a.double().flatten(), b.double().flatten()
    return (a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item()


@pytest.mark.parametrize("model_name", ["resnet18", "efficientnet-b0"])
def test_grad_arena(model_name):
    """Backward kernels write gradients straight into the persistent arena slots: same values as
    freshly allocated gradients, every .grad aliases its slot, a second backward without begin()
    accumulates, and the fused Adam pointer table is built once across steps.

    Compared by per-parameter cosine similarity: fp32-atomic ordering (BN statistics, split-K) is
    not bitwise reproducible and small BatchNorm populations amplify one-ulp bf16 flips: EfficientNet
    at random init is chaotic in train mode (BN gradient explosion at init), so it runs in eval mode."""
    from pytorch_imageclassification_distributed_amd.engine.optim import FusedAdam
    from pytorch_imageclassification_distributed_amd.models import Classifier
    from pytorch_imageclassification_distributed_amd.ops.grad_arena import GradArena
    torch.manual_seed(0)
    m = Classifier(model_name, 5).to(DEV).to(memory_format=torch.channels_last).train()
    if model_name.startswith("efficientnet"):
        m.eval()  # train-mode EfficientNet at init is chaotic run to run (see above); eval is reproducible
    x = torch.randn(8, 3, 128, 128, device=DEV)
    params = [p for p in m.parameters() if p.requires_grad]
    names = [n for n, p in m.named_parameters() if p.requires_grad]

    same = _SameState(m)

    def loss_fn():
        same()
        torch.manual_seed(1)  # same dropout / drop-connect masks every call
        return m(x).float().square().mean()

    def check(got, want, what):
        big = max(w.norm().item() for w in want)
        for n, g_, w in zip(names, got, want):
            if w.norm().item() > 1e-3 * big:
                assert _cos(g_, w) > 0.995, (what, n, _cos(g_, w))
                assert abs(g_.norm().item() / w.norm().item() - 1) < 0.03, (what, n)

    loss_fn().backward()  # no arena: fresh tensors
    ref = [p.grad.clone() for p in params]
    arena = GradArena(params, list(reversed(range(len(params)))))
    for p in params:
        p.grad = None
    arena.begin()
    loss_fn().backward()
    assert all(arena.owns(p) for p in params), [n for n, p in m.named_parameters() if not arena.owns(p)]
    check([p.grad for p in params], ref, "arena vs fresh")
    one = [p.grad.clone() for p in params]
    loss_fn().backward()  # accumulation without re-arming: slot += new gradient
    assert all(arena.owns(p) for p in params)
    check([p.grad for p in params], [2 * o for o in one], "accumulate")
    opt = FusedAdam(params, lr=1e-4)
    keys = set()
    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        arena.begin()
        loss_fn().backward()
        opt.step()
        keys.add(opt._table_key)
    assert len(keys) == 1
    torch.cuda.synchronize()


@pytest.mark.parametrize("model_name", ["resnet18", "efficientnet-b0"])
def test_deterministic_mode(model_name):
    """set_deterministic(True): two identical fwd+bwd passes give bitwise-equal outputs and gradients
    (train mode, BN batch statistics, drop-connect, split-K sites all reorganised), and the result
    agrees with the default (atomic-order) mode to rounding."""
    from pytorch_imageclassification_distributed_amd.models import Classifier
    from pytorch_imageclassification_distributed_amd.ops import hip
    torch.manual_seed(0)
    m = Classifier(model_name, 5).to(DEV).to(memory_format=torch.channels_last).train()
    x = torch.randn(4, 3, 96, 96, device=DEV)
    same = _SameState(m)

    def run():
        same()
        for p in m.parameters():
            p.grad = None
        torch.manual_seed(1)
        out = m(x).float()
        out.square().mean().backward()
        return out.detach().clone(), [p.grad.clone() for p in m.parameters()]

    hip.set_deterministic(True)
    try:
        o1, g1 = run()
        o2, g2 = run()
    finally:
        hip.set_deterministic(False)
    assert torch.equal(o1, o2)
    for a, b in zip(g1, g2):
        assert torch.equal(a, b)
    o3, _ = run()
    torch.testing.assert_close(o3, o1, rtol=0.05, atol=0.05 * o1.abs().max().item())


@pytest.mark.parametrize("model_name", ["resnet50", "inceptionv3"])
def test_wgrad_side_stream(model_name):
    """Weight gradients on the side stream (arena slots) are bitwise the single-stream ones in
    deterministic mode, over three steps with begin() / Adam in between: the side stream starts
    behind the arena memset, its inputs outlive their autograd lifetime (record_stream), and the
    compute stream joins it before anything reads a gradient."""
    from pytorch_imageclassification_distributed_amd.engine.optim import FusedAdam
    from pytorch_imageclassification_distributed_amd.models import Classifier
    from pytorch_imageclassification_distributed_amd.ops import hip
    from pytorch_imageclassification_distributed_amd.ops.grad_arena import GradArena

    def run(side):
        torch.manual_seed(0)
        m = Classifier(model_name, 7).to(DEV).to(memory_format=torch.channels_last).train()
        params = [p for p in m.parameters() if p.requires_grad]
        arena = GradArena(params, list(reversed(range(len(params)))))
        opt = FusedAdam(params, lr=1e-3)
        hw = 96 if model_name == "resnet50" else 299
        x = torch.randn(4, 3, hw, hw, device=DEV)
        hip.WGRAD_STREAM = side
        out = []
        for _ in range(3):
            opt.zero_grad(set_to_none=True)
            arena.begin()
            torch.manual_seed(1)
            y = m(x)
            y = sum(t.float().square().mean() for t in y) if isinstance(y, tuple) else y.float().square().mean()
            y.backward()
            out.append([p.grad.clone() for p in params])
            opt.step()
        return out, [p.detach().clone() for p in params]

    keep = hip.WGRAD_STREAM
    hip.set_deterministic(True)
    try:
        g_side, p_side = run(True)
        assert hip._SIDE, "side stream never used"
        g_one, p_one = run(False)
    finally:
        hip.set_deterministic(False)
        hip.WGRAD_STREAM = keep
    for step, (a_, b_) in enumerate(zip(g_side, g_one)):
        for i, (a, b) in enumerate(zip(a_, b_)):
            assert torch.equal(a, b), (step, i)
    for a, b in zip(p_side, p_one):
        assert torch.equal(a, b)


@pytest.mark.parametrize("kind,expect", [("A", 3), ("B", 2), ("C", 6), ("D", 4), ("E", 3)])
def test_inception_block_fusion(kind, expect):
    """Inception blocks: chain-internal convs fuse their producer's BN-backward reduce and InceptionE's
    paired slots fuse too; gradients equal the unfused path."""
    from pytorch_imageclassification_distributed_amd.models import inception as inc
    from pytorch_imageclassification_distributed_amd.ops import hip
    torch.manual_seed(0)
    blk, cin, hw = {"A": (inc.InceptionA(64, 32), 64, 17), "B": (inc.InceptionB(64), 64, 17),
                    "C": (inc.InceptionC(128, 64), 128, 9), "D": (inc.InceptionD(128), 128, 9),
                    "E": (inc.InceptionE(128), 128, 8)}[kind]
    blk = blk.to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(4, cin, hw, hw, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    keep_sib, hip.SIBLINGS = hip.SIBLINGS, False  # (the per-branch path: merged sibling heads take no consumer reduce)
    try:
        gx0, gp0 = _grads(blk, x, False)
        before = hip.FUSED_BWD_COUNT[0]
        gx1, gp1 = _grads(blk, x, True)
    finally:
        hip.SIBLINGS = keep_sib
    assert hip.FUSED_BWD_COUNT[0] - before == expect
    err = lambda a, b: ((a - b).abs().max() / b.abs().max().clamp(min=1e-6)).item()  # noqa: E731
    assert err(gx1, gx0) < 3e-2, err(gx1, gx0)
    for n in gp0:
        assert err(gp1[n], gp0[n]) < 3e-2, (n, err(gp1[n], gp0[n]))


@pytest.mark.parametrize("kind", ["A", "B", "C", "D", "E"])
def test_inception_concat_in_place(kind):
    """Inception blocks: branches writing their BN output straight into the concat buffer (and reading
    their gradient slices in place) == copying branches into a fresh concat (forward and gradients)."""
    from pytorch_imageclassification_distributed_amd.models import inception as I
    from pytorch_imageclassification_distributed_amd.ops import hip
    torch.manual_seed(0)
    blk, cin, hw = {"A": (I.InceptionA(192, 32), 192, 17), "B": (I.InceptionB(288), 288, 17),
                    "C": (I.InceptionC(768, 128), 768, 9), "D": (I.InceptionD(768), 768, 9),
                    "E": (I.InceptionE(1280), 1280, 5)}[kind]
    blk = blk.to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(4, cin, hw, hw, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    same = _SameState(blk)

    def run(inplace):
        same()
        keep, hip.CONCAT_INPLACE = hip.CONCAT_INPLACE, inplace
        try:
            for p in blk.parameters():
                p.grad = None
            xx = x.clone().requires_grad_(True)
            out = blk(xx)
            (out.float() * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum().backward()
            return out.float(), xx.grad.float(), {n: p.grad.float().clone() for n, p in blk.named_parameters()}
        finally:
            hip.CONCAT_INPLACE = keep

    o0, gx0, gp0 = run(False)
    o1, gx1, gp1 = run(True)
    err = lambda a, b: ((a - b).abs().max() / b.abs().max().clamp(min=1e-6)).item()  # noqa: E731
    assert err(o1, o0) < 1e-2
    assert err(gx1, gx0) < 2e-2, err(gx1, gx0)
    for n in gp0:
        assert err(gp1[n], gp0[n]) < 2e-2, (n, err(gp1[n], gp0[n]))


@pytest.mark.parametrize("kind", ["A", "C", "E"])
def test_inception_pool_conv_swap(kind):
    """Inception branch_pool: the HIP path's conv1x1 -> avgpool order (conv on the wide input, pool on
    the narrow output) against the fp32 torch reference's avgpool -> conv1x1, forward and gradients -
    and no further from it than the HIP path with the pool first (the bf16 block's own error level)."""
    from pytorch_imageclassification_distributed_amd.models import inception as I
    from pytorch_imageclassification_distributed_amd.ops import functional as Fx
    from pytorch_imageclassification_distributed_amd.ops import hip
    torch.manual_seed(1)
    blk, cin, hw = {"A": (I.InceptionA(192, 32), 192, 17), "C": (I.InceptionC(768, 128), 768, 9),
                    "E": (I.InceptionE(1280), 1280, 5)}[kind]
    blk = blk.to(DEV).to(memory_format=torch.channels_last)
    with torch.no_grad():
        for p in blk.parameters():
            p.copy_(p.to(torch.bfloat16).float())
    x = torch.randn(4, cin, hw, hw, device=DEV).to(torch.bfloat16).float()
    wgt = None

    def run(swap, backend="auto"):
        nonlocal wgt
        m = copy.deepcopy(blk)
        keep_b, keep_s = Fx.get_backend(), hip.POOL_CONV_SWAP
        Fx.set_backend(backend)
        hip.POOL_CONV_SWAP = swap
        try:
            xx = (x.clone() if backend == "torch" else
                  x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)).requires_grad_(True)
            out = m(xx)
            if wgt is None:
                wgt = torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)
            (out.float() * wgt).sum().backward()
            return out.float(), xx.grad.float(), {n: p.grad.float() for n, p in m.named_parameters()}
        finally:
            Fx.set_backend(keep_b)
            hip.POOL_CONV_SWAP = keep_s

    o_r, gx_r, gp_r = run(False, "torch")
    o_s, gx_s, gp_s = run(True)
    o_p, gx_p, gp_p = run(False)
    err = lambda a, b: ((a - b).abs().max() / b.abs().max().clamp(min=1e-6)).item()  # noqa: E731
    merr = lambda a, b: ((a - b).abs().mean() / b.abs().mean().clamp(min=1e-9)).item()  # noqa: E731
    assert err(o_s, o_r) < 3e-2
    assert merr(gx_s, gx_r) < max(3e-2, 1.3 * merr(gx_p, gx_r)), (merr(gx_s, gx_r), merr(gx_p, gx_r))
    for n in gp_r:
        if "branch_pool" in n:
            assert merr(gp_s[n], gp_r[n]) < max(3e-2, 1.3 * merr(gp_p[n], gp_r[n])), n


@pytest.mark.parametrize("kind,fp8", [("bottle_id", False), ("chain", False), ("chain", True)])
def test_relu_mask_matches_residual_recompute(kind, fp8):
    """The residual BN's forward ReLU mask (bn_apply writes 1 bit per element; the consuming conv's dgrad
    epilogue reads it instead of re-reading the residual) gives the gradients of the recompute path."""
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.models.resnet import Bottleneck, _conv1x1
    from pytorch_imageclassification_distributed_amd.ops import hip
    torch.manual_seed(0)
    if kind == "bottle_id":
        blk = nn.Sequential(Bottleneck(256, 64), Bottleneck(256, 64))
    else:
        blk = nn.Sequential(Bottleneck(256, 128, 2, nn.Sequential(_conv1x1(256, 512, 2), nn.BatchNorm2d(512))),
                            Bottleneck(512, 128))
    blk = blk.to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(4, 256, 16, 16, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    keep = hip.RELU_MASK
    hip.set_fp8(fp8)  # fp8: the residual BN writes its mask from the MX-FP8 apply kernel
    try:
        hip.RELU_MASK = False
        gx0, gp0 = _grads(blk, x, True)
        hip.RELU_MASK = True
        gx1, gp1 = _grads(blk, x, True)
    finally:
        hip.RELU_MASK = keep
        hip.set_fp8(False)
    err = lambda a, b: ((a - b).abs().max() / b.abs().max().clamp(min=1e-6)).item()  # noqa: E731
    assert err(gx1, gx0) < 1e-2, err(gx1, gx0)
    for n in gp0:
        assert err(gp1[n], gp0[n]) < 1e-2, (n, err(gp1[n], gp0[n]))


@pytest.mark.parametrize("n_blocks,hw", [(2, 16), (1, 15)])
def test_fused_xa_backward_matches_separate(n_blocks, hw):
    """conv_fused_bwd_kernel (ResNet layer1 conv3: 64 -> 256) and conv_fused_bwd_n_kernel (conv1: 256 -> 64, the
    residual gradient as the dgrad addend), XA: one pass over dz and y gives the data gradient with its
    BN-backward epilogue and the weight gradient - the same values as the separate XA dgrad and XA wgrad
    launches (odd map: partial last pixel tile)."""
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.models.resnet import Bottleneck
    from pytorch_imageclassification_distributed_amd.ops import hip
    torch.manual_seed(0)
    blk = nn.Sequential(*[Bottleneck(256, 64) for _ in range(n_blocks)]).to(DEV).to(memory_format=torch.channels_last)
    x = torch.randn(4, 256, hw, hw, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    keep, keep_n = hip.FUSED_XA_BWD, hip.FUSED_XA_BWD_N
    hip.FUSED_XA_BWD_N = True  # both fused forms (the 64-output one is off by default)
    try:
        hip.FUSED_XA_BWD = False
        gx0, gp0 = _grads(blk, x, True)
        hip.FUSED_XA_BWD = True
        before = hip.FUSED_XA_BWD_COUNT[0]
        gx1, gp1 = _grads(blk, x, True)
        assert hip.FUSED_XA_BWD_COUNT[0] - before == 2 * n_blocks  # conv1 (256 -> 64) and conv3 (64 -> 256)
    finally:
        hip.FUSED_XA_BWD, hip.FUSED_XA_BWD_N = keep, keep_n
    err = lambda a, b: ((a - b).abs().max() / b.abs().max().clamp(min=1e-6)).item()  # noqa: E731
    assert err(gx1, gx0) < 1e-2, err(gx1, gx0)
    for n in gp0:
        assert err(gp1[n], gp0[n]) < 1e-2, (n, err(gp1[n], gp0[n]))


@pytest.mark.parametrize("kind", ["basic_ds", "bottle_ds", "chain", "chain_bigmean"])
@pytest.mark.parametrize("fused", [True, False])
def test_deferred_downsample_bn(kind, fused):
    """The downsample BN's apply folded into the residual BN's (ops/_hip/convbn.py RES_DEFER: the residual
    apply forms sc3 * y3 + sh3 + bf16(sc_ds * y_ds + sh_ds)): input and parameter gradients and running
    statistics equal the materialized residual's, with the fused BN backward on (the consumer reads the ReLU
    mask) and off (the residual BN's backward re-forms the residual).  The output also matches in eval mode
    (not deferred).  In the chain the next block's conv1 data-gradient epilogue also accumulates the downsample
    BN's backward partial sums (``BwdLink.ds``)."""
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.models.resnet import BasicBlock, Bottleneck, _conv1x1
    from pytorch_imageclassification_distributed_amd.ops import hip
    torch.manual_seed(1)
    if kind == "basic_ds":
        blk, cin = BasicBlock(64, 128, 2, nn.Sequential(_conv1x1(64, 128, 2), nn.BatchNorm2d(128))), 64
    elif kind == "bottle_ds":
        blk, cin = Bottleneck(256, 128, 2, nn.Sequential(_conv1x1(256, 512, 2), nn.BatchNorm2d(512))), 256
    else:
        blk = nn.Sequential(Bottleneck(256, 128, 2, nn.Sequential(_conv1x1(256, 512, 2), nn.BatchNorm2d(512))),
                            Bottleneck(512, 128))
        cin = 256
    shift = 0.0
    if kind == "chain_bigmean":
        # the downsample conv's output channels with |mean| / std ~ 30: the second-BN partial sums of the fused
        # epilogue (sum dz * (y_ds - mean_ds)) must not cancel (centred per element, not per block)
        with torch.no_grad():
            blk[0].downsample[0].weight.add_(0.05)
        shift = 3.0
    blk = blk.to(DEV).to(memory_format=torch.channels_last)
    ref = copy.deepcopy(blk)
    x = (torch.randn(4, cin, 16, 16, device=DEV) + shift).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    keep = hip.RES_DEFER
    try:
        hip.RES_DEFER = False
        gx0, gp0 = _grads(ref, x, fused)
        hip.RES_DEFER = True
        n0, d0 = hip.RES_DEFER_COUNT[0], hip.DS_FUSE_COUNT[0]
        gx1, gp1 = _grads(blk, x, fused)
        # (IMGCLS_BN_WALK / unroll A/B knobs can leave bn_apply without its residual-coefficient form: the
        # residual is then materialised, and the results below must still match)
        if hip.C.bn_res_coef_ok(True):
            assert hip.RES_DEFER_COUNT[0] > n0, "the downsample BN was not deferred"
        if kind.startswith("chain") and fused and hip.DS_FUSE:
            # the second block's conv1 data gradient produced the first block's dz: it took the downsample BN's
            # partial sums too (gemm.DS_FUSE)
            assert hip.DS_FUSE_COUNT[0] > d0, "the downsample BN's partial sums did not ride in the epilogue"
    finally:
        hip.RES_DEFER = keep
    err = lambda a, b: ((a - b).abs().max() / b.abs().max().clamp(min=1e-6)).item()  # noqa: E731
    assert err(gx1, gx0) < 1e-2, err(gx1, gx0)
    for n in gp0:
        assert err(gp1[n], gp0[n]) < 1e-2, (n, err(gp1[n], gp0[n]))
    for (n, b0), b1 in zip(ref.named_buffers(), blk.buffers()):
        if b0.is_floating_point():
            assert torch.allclose(b1, b0, rtol=1e-3, atol=1e-4), n
    blk.eval()
    ref.eval()
    with torch.no_grad():
        assert err(blk(x).float(), ref(x).float()) < 1e-2


def _bn_fin_run(hip, fn, x, mods, fin):
    """One forward + backward with IMGCLS_BN_FIN set to ``fin``: (output, input grad, param grads, buffers, fused
    BN count).  Buffers are restored first (running stats are the statistics pivot)."""
    keep, keep_bwd = hip.BN_FIN, hip.BN_FIN_BWD
    hip.BN_FIN = hip.BN_FIN_BWD = fin
    try:
        for m in mods:
            m._imgcls_same_state = getattr(m, "_imgcls_same_state", None) or _SameState(m)
            m._imgcls_same_state()
            for p in m.parameters():
                p.grad = None
        n0 = hip.BN_FIN_COUNT[0] + 1000 * hip.BN_FIN_BWD_COUNT[0]
        xx = x.clone().requires_grad_(True)
        out = fn(xx)
        (out.float() * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum().backward()
        torch.cuda.synchronize()
        grads = [p.grad.float().clone() for m in mods for p in m.parameters()]
        bufs = [b.detach().clone() for m in mods for b in m.buffers()]
        return (out.float(), xx.grad.float(), grads, bufs,
                hip.BN_FIN_COUNT[0] + 1000 * hip.BN_FIN_BWD_COUNT[0] - n0)
    finally:
        hip.BN_FIN, hip.BN_FIN_BWD = keep, keep_bwd


@pytest.mark.parametrize("kind", ["inception_a", "silu_136", "none_80"])
def test_bn_fin_apply_matches_two_launch_path(kind):
    """BN_FIN (the training BN's partial-row reduce and finalize inside its apply kernel, csrc/bn.hip
    bn_fin_apply_kernel, and the backward reduce inside the elementwise pass, bn_fin_bwd_kernel) against the
    separate launches: outputs (incl. concat slices), running statistics,
    batch counters and every gradient.  Two fused runs in a row must agree: the kernel's last block per channel
    chunk re-zeroes the partial rows and resets its counter, or the second run would double-count."""
    import torch.nn as nn
    from pytorch_imageclassification_distributed_amd.models.inception import InceptionA
    from pytorch_imageclassification_distributed_amd.ops import hip
    CL = torch.channels_last
    torch.manual_seed(0)
    if kind == "inception_a":  # 64 / 48 / 96 / 32-channel BNs writing concat slices, 35 x 35 -> 11 x 11 here
        blk = InceptionA(192, 32).to(DEV).to(memory_format=CL).train()
        mods, fn = [blk], blk
        x = torch.randn(2, 192, 11, 11, device=DEV).to(torch.bfloat16).contiguous(memory_format=CL)
    else:
        c, act = (136, "silu") if kind == "silu_136" else (80, None)  # a partial 64-channel chunk
        conv = nn.Conv2d(32, c, 1, bias=False).to(DEV).to(memory_format=CL)
        bn = nn.BatchNorm2d(c).to(DEV)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
            bn.running_mean.uniform_(-0.2, 0.2)
        mods = [conv, bn]
        fn = lambda t: hip.conv_bn_act(t, conv, bn, act, None)  # noqa: E731
        x = torch.randn(3, 32, 13, 13, device=DEV).to(torch.bfloat16).contiguous(memory_format=CL)
    ref = _bn_fin_run(hip, fn, x, mods, False)
    f1 = _bn_fin_run(hip, fn, x, mods, True)
    f2 = _bn_fin_run(hip, fn, x, mods, True)
    assert ref[4] == 0 and f1[4] % 1000 > 0 and f1[4] >= 1000 and f1[4] == f2[4]  # forward and backward fused
    for r in (f1, f2):
        assert (r[0] - ref[0]).abs().max().item() <= 1e-2 * ref[0].abs().max().item()
        assert (r[1] - ref[1]).abs().max().item() <= 1e-2 * ref[1].abs().max().item() + 1e-6
        for a_, b_ in zip(r[2], ref[2]):
            assert (a_ - b_).abs().max().item() <= 1e-2 * b_.abs().max().item() + 1e-6
        for a_, b_ in zip(r[3], ref[3]):
            assert torch.allclose(a_.float(), b_.float(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("kind", ["A", "C", "D", "E"])
def test_inception_sibling_heads_merged(kind):
    """The 1x1 heads of an Inception block as one concatenated-output GEMM with per-slice BN (ops/_hip/convbn.py
    SiblingConvFn / SiblingBNFn) == the per-branch path: block output, input gradient, every parameter gradient,
    the BN running statistics and batch counters."""
    from pytorch_imageclassification_distributed_amd.models import inception as inc
    from pytorch_imageclassification_distributed_amd.ops import hip
    torch.manual_seed(0)
    blk, cin, hw = {"A": (inc.InceptionA(192, 32), 192, 11), "C": (inc.InceptionC(256, 64), 256, 9),
                    "D": (inc.InceptionD(256), 256, 9), "E": (inc.InceptionE(256), 256, 5)}[kind]
    blk = blk.to(DEV).to(memory_format=torch.channels_last).train()
    with torch.no_grad():
        for m in blk.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.5, 0.5)
                m.running_mean.uniform_(-0.2, 0.2)
    x = torch.randn(4, cin, hw, hw, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    same = _SameState(blk)

    def run(merged):
        keep, hip.SIBLINGS = hip.SIBLINGS, merged
        try:
            same()
            for p in blk.parameters():
                p.grad = None
            n0 = hip.SIBLINGS_COUNT[0]
            xx = x.clone().requires_grad_(True)
            out = blk(xx)
            (out.float() * torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out)).sum().backward()
            torch.cuda.synchronize()
            return (out.float(), xx.grad.float(), {n: p.grad.float().clone() for n, p in blk.named_parameters()},
                    [b.detach().float().clone() for b in blk.buffers()], hip.SIBLINGS_COUNT[0] - n0)
        finally:
            hip.SIBLINGS = keep

    ref, mrg = run(False), run(True)
    assert ref[4] == 0 and mrg[4] == 1
    err = lambda a, b: ((a - b).abs().max() / b.abs().max().clamp(min=1e-6)).item()  # noqa: E731
    assert err(mrg[0], ref[0]) < 2e-2, err(mrg[0], ref[0])
    assert err(mrg[1], ref[1]) < 3e-2, err(mrg[1], ref[1])
    for n in ref[2]:
        assert err(mrg[2][n], ref[2][n]) < 3e-2, (n, err(mrg[2][n], ref[2][n]))
    for a, b in zip(mrg[3], ref[3]):
        assert torch.allclose(a, b, rtol=1e-3, atol=1e-4)
