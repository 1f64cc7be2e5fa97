"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

Inputs are rounded to bf16 first (the HIP path stores activations/weights in
bf16), the reference then runs in fp32 on those exact values, so the remaining
error is the kernels' fp32-accumulation order plus the bf16 rounding of outputs.
"""
import copy
import math

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
CL = torch.channels_last


def _hip():
    from pytorch_imageclassification_distributed_amd.ops import hip
    return hip


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / b.abs().max().clamp(min=1e-6)).item()


def mean_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().mean() / b.abs().mean().clamp(min=1e-9)).item()


def bf(x):
    return x.to(torch.bfloat16).float()


CONV_CASES = [
    # N, Cin, H, W, Cout, k, stride, pad
    (2, 64, 56, 56, 64, (1, 1), 1, (0, 0)),
    (2, 64, 56, 56, 64, (3, 3), 1, (1, 1)),
    (2, 64, 56, 56, 256, (1, 1), 1, (0, 0)),
    (2, 128, 56, 56, 128, (3, 3), 2, (1, 1)),
    (2, 256, 56, 56, 512, (1, 1), 2, (0, 0)),
    (2, 512, 7, 7, 2048, (1, 1), 1, (0, 0)),
    (3, 512, 7, 7, 512, (3, 3), 1, (1, 1)),
    (2, 8, 64, 64, 64, (7, 7), 2, (3, 3)),
    (2, 64, 17, 17, 64, (1, 7), 1, (0, 3)),
    (2, 64, 17, 17, 96, (7, 1), 1, (3, 0)),
    (2, 48, 35, 35, 64, (5, 5), 1, (2, 2)),
    (2, 96, 35, 35, 96, (3, 3), 2, (0, 0)),
    (1, 32, 15, 13, 40, (3, 3), 1, (0, 0)),
    (2, 32, 37, 37, 32, (3, 3), 1, (0, 0)),   # 32-row wgrad tile (Inception Conv2d_2a)
    (2, 24, 20, 20, 24, (3, 3), 1, (1, 1)),   # ... with a partial 24-of-32 channel tile (EfficientNet widths)
    (2, 24, 20, 20, 144, (1, 1), 1, (0, 0)),  # EfficientNet expand 1x1: Ntot 24 (a partial 64-column wgrad tile)
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_bwd(case):
    hip = _hip()
    n, cin, h, w, cout, k, s, p = case
    torch.manual_seed(0)
    conv = nn.Conv2d(cin, cout, k, s, p, bias=False).to(DEV).to(memory_format=CL)
    with torch.no_grad():
        conv.weight.copy_(bf(conv.weight))
    x = bf(torch.randn(n, cin, h, w, device=DEV)).contiguous(memory_format=CL)
    xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    y = hip.ConvFn.apply(xb, conv.weight, conv, False)
    xr = x.clone().requires_grad_(True)
    wr = conv.weight.detach().clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, s, p)
    assert y.shape == yr.shape
    assert rel_err(y, yr) < 1e-2
    gy = bf(torch.randn_like(yr))
    y.backward(gy.to(torch.bfloat16).contiguous(memory_format=CL))
    yr.backward(gy)
    assert rel_err(xb.grad, xr.grad) < 2e-2
    assert rel_err(conv.weight.grad, wr.grad) < 2e-2


def _table_len(name, default):
    """Length of a kernel configuration table, read from the built extension at collection time so
    the parametrisation is exact; without the extension fall back to an upper bound (indices past the
    table then skip)."""
    try:
        return len(getattr(_hip(), name)())
    except Exception:  # extension not built / not importable here
        return default


N_CFG = _table_len("conv_cfgs", 24)
N_FP8_CFG = _table_len("conv_fp8_cfgs", 8)


def _wgrad_stage_ok(case, stages):
    # stages 4 / 7 / 9 = 256x256 8-wave tile (Cout >= 256), 5/6 = 32-row tile (Cout <= 32), 8 = any,
    # 10 / 11 = 64-column tiles (any), 12 = 256 x 64 (Cout >= 256)
    return not ((stages in (4, 7, 9, 12) and case[4] < 256) or (stages in (5, 6) and case[4] > 32)
                or (stages == 16 and case[4] > 64))


@pytest.mark.parametrize("cfg", range(N_CFG))
@pytest.mark.parametrize("case", [CONV_CASES[1], CONV_CASES[2], CONV_CASES[3], CONV_CASES[6], CONV_CASES[7],
                                  CONV_CASES[10], CONV_CASES[12]])
def test_conv_tile_configs(case, cfg):
    """Every entry of the kernel configuration table the per-shape tuner can pick (tile rows x
    channels, wave layout, ring depth) matches the fp32 reference (fwd, dgrad phases)."""
    hip = _hip()
    if cfg >= len(hip.conv_cfgs()):
        pytest.skip("past the configuration table")
    keep, hip.CONV_FORCE_CFG = hip.CONV_FORCE_CFG, (0, 0, cfg)
    try:
        test_conv_fwd_bwd(case)
    finally:
        hip.CONV_FORCE_CFG = keep


N_HALO = _table_len("conv_halo_cfgs", 12)
HALO_CASES = [
    CONV_CASES[1],                             # 64 ch, 56 x 56 (W = 56: the 384-row patches only)
    CONV_CASES[6],                             # 512 ch, 7 x 7: a tile spans many images
    (2, 128, 15, 13, 128, (3, 3), 1, (1, 1)),  # odd map: rows wrap mid-tile, partial last tile
    (2, 128, 28, 28, 96, (3, 3), 1, (1, 1)),   # partial output-channel tile
    (2, 64, 8, 8, 64, (1, 3), 1, (0, 1)),      # Inception 1x3 (3 taps in a row)
    (2, 64, 8, 8, 64, (3, 1), 1, (1, 0)),      # ... and 3x1
]


@pytest.mark.parametrize("cfg", range(N_HALO))
@pytest.mark.parametrize("case", HALO_CASES)
def test_conv_halo_configs(case, cfg):
    """Every halo-patch configuration (csrc/conv_halo.hip) forced on the stride-1 3x3-window convs it
    accepts: forward and the stride-1 data gradient against the fp32 reference, and the kernel ran."""
    hip = _hip()
    if cfg >= len(hip.conv_halo_cfgs()):
        pytest.skip("past the configuration table")
    keep, hip.HALO_FORCE = hip.HALO_FORCE, cfg
    before = hip.HALO_COUNT[0]
    try:
        test_conv_fwd_bwd(case)
    finally:
        hip.HALO_FORCE = keep
    tm, pmax, w = hip.conv_halo_cfgs()[cfg][0], hip.conv_halo_cfgs()[cfg][5], case[3]
    if tm + 2 * w + 2 <= pmax:  # the data gradient (K = taps x Cout) qualifies when Cout % 64 == 0
        expect = 1 + (case[4] % 64 == 0)
        assert hip.HALO_COUNT[0] - before >= expect, "halo kernel not launched"


N_DEEP = _table_len("conv_deep_cfgs", 12)
DEEP_CASES = [CONV_CASES[i] for i in (0, 1, 2, 3, 4, 5, 6)] + [
    (2, 128, 15, 13, 128, (3, 3), 1, (1, 1)),  # odd map: partial last row tile
    (2, 128, 28, 28, 96, (3, 3), 1, (1, 1)),   # partial output-channel tile
    (1, 64, 9, 9, 320, (3, 3), 2, (1, 1)),     # stride 2, partial column tile of a 256-wide tile
]


@pytest.mark.parametrize("cfg", range(N_DEEP))
@pytest.mark.parametrize("case", DEEP_CASES)
def test_conv_deep_configs(case, cfg):
    """Every prefetch-depth-2 configuration (csrc/conv_deep.hip) forced on each launch it accepts (64-channel
    k-steps): forward and data-gradient phases against the fp32 reference, and the kernel ran."""
    hip = _hip()
    if cfg >= len(hip.conv_deep_cfgs()) or hip.conv_deep_cfgs()[cfg][4] & 6:
        pytest.skip("past the configuration table / a diagnostic variant")
    keep, hip.DEEP_FORCE = hip.DEEP_FORCE, cfg
    before = hip.DEEP_COUNT[0]
    try:
        test_conv_fwd_bwd(case)
    finally:
        hip.DEEP_FORCE = keep
    assert hip.DEEP_COUNT[0] - before >= 1 + (case[4] % 64 == 0), "deep kernel not launched"


@pytest.mark.parametrize("cfg", range(N_DEEP))
@pytest.mark.parametrize("act,use_res", [("relu", True), ("silu", False)])
def test_conv_bn_act_deep(act, use_res, cfg):
    """Fused epilogues (BN statistics, residual, BN-backward link) on every prefetch-depth-2 configuration."""
    hip = _hip()
    if cfg >= len(hip.conv_deep_cfgs()) or hip.conv_deep_cfgs()[cfg][4] & 6:
        pytest.skip("past the configuration table / a diagnostic variant")
    keep, hip.DEEP_FORCE = hip.DEEP_FORCE, cfg
    before = hip.DEEP_COUNT[0]
    try:
        test_conv_bn_act(act, use_res)
    finally:
        hip.DEEP_FORCE = keep
    assert hip.DEEP_COUNT[0] > before


@pytest.mark.parametrize("cfg", range(N_DEEP))
@pytest.mark.parametrize("mnk", [(4096 + 40, 512, 1024), (700, 200, 192), (20000, 2048, 64)])
def test_conv_deep_plain_gemm(mnk, cfg):
    """The GEMM view (benchmarks/gemm_ref.py: a 1x1 conv over an M x 1 'image', so the input height exceeds
    the kernel's 16-bit coordinates) against torch.mm in fp32: partial row / column tiles, K of 1..16 steps."""
    hip = _hip()
    if cfg >= len(hip.conv_deep_cfgs()) or hip.conv_deep_cfgs()[cfg][4] & 6:
        pytest.skip("past the configuration table / a diagnostic variant")
    M, N, K = mnk
    torch.manual_seed(0)
    A = (torch.rand(M, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=DEV) * 2 - 1).to(torch.bfloat16)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    geo = (M, N, K, K, M, 1, M, 1, 1, K, M, 1, 1, 0, 0, N, 0)
    hip.C.conv_gemm(A, B.view(-1), out, None, None, *geo, [0], [0], [0], hip.G_STATS, hip.ws(torch.device(DEV)).zero,
                    None, None, None, None, None, 0, 1, 0, 0, hip.DEEP_BASE + cfg, None, None, None, None, None, None,
                    None, 0, None, None, None, None, 0)
    ref = A.float() @ B.float().t()
    assert torch.isfinite(out.float()).all()
    assert rel_err(out, ref) < 1e-2


N_PW = _table_len("conv_pw_cfgs", 12)
PW_CASES = [  # N, Cin, H, W, Cout: EfficientNet expand / project 1x1 shapes, partial fragments and channel tiles
    (2, 16, 40, 40, 96), (2, 24, 28, 28, 144), (3, 144, 20, 20, 24), (2, 32, 33, 31, 16), (2, 40, 14, 14, 240),
    (2, 96, 15, 15, 24), (1, 80, 9, 7, 48)]


@pytest.mark.parametrize("cfg", range(N_PW))
@pytest.mark.parametrize("case", PW_CASES)
def test_conv_pw_configs(case, cfg):
    """Every register-resident-weight pointwise configuration (csrc/conv_pw.hip) forced on the 1x1 forward it
    covers, inside conv -> BN (train) -> SiLU: output (through the epilogue's BN statistics), running
    statistics and the backward against fp32 torch, and the kernel ran."""
    hip = _hip()
    if cfg >= len(hip.conv_pw_cfgs()):
        pytest.skip("past the configuration table")
    n, c, h, w, co = case
    if c > hip.conv_pw_cfgs()[cfg][1]:
        pytest.skip("K exceeds the entry's k capacity")
    torch.manual_seed(3)
    conv = nn.Conv2d(c, co, 1, bias=False).to(DEV).to(memory_format=CL)
    bn = nn.BatchNorm2d(co).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(bf(conv.weight))
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.2, 0.2)  # a non-zero statistics pivot (the BN's running mean)
    conv_r = nn.Conv2d(c, co, 1, bias=False).to(DEV)
    bn_r = nn.BatchNorm2d(co).to(DEV)
    conv_r.load_state_dict(conv.state_dict())
    bn_r.load_state_dict(bn.state_dict())
    x = bf(torch.randn(n, c, h, w, device=DEV))
    xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    keep, hip.PW_FORCE = hip.PW_FORCE, cfg
    before = hip.PW_COUNT[0]
    try:
        out = hip.conv_bn_act(xb, conv, bn, "silu", None)
    finally:
        hip.PW_FORCE = keep
    assert hip.PW_COUNT[0] > before, "pointwise kernel not launched"
    xr = x.clone().requires_grad_(True)
    yc = conv_r(xr)
    yc = yc + (bf(yc) - yc).detach()
    ref = F.silu(bn_r(yc))
    assert rel_err(out, ref) < 2e-2
    assert torch.allclose(bn.running_mean, bn_r.running_mean, rtol=1e-2, atol=1e-3)
    assert torch.allclose(bn.running_var, bn_r.running_var, rtol=1e-2, atol=1e-3)
    g = bf(torch.randn_like(ref))
    out.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
    torch.cuda.synchronize()  # a fault in this backward's kernels is reported here, not inside the reference's
    ref.backward(g)
    assert rel_err(xb.grad, xr.grad) < 3e-2
    assert rel_err(conv.weight.grad, conv_r.weight.grad) < 3e-2


@pytest.mark.parametrize("cfg", range(N_HALO))
@pytest.mark.parametrize("act,use_res", [("relu", True), ("silu", False)])
def test_conv_bn_act_halo(act, use_res, cfg):
    """Fused epilogues (BN statistics, residual, BN-backward link) on every halo configuration."""
    hip = _hip()
    if cfg >= len(hip.conv_halo_cfgs()):
        pytest.skip("past the configuration table")
    keep, hip.HALO_FORCE = hip.HALO_FORCE, cfg
    before = hip.HALO_COUNT[0]
    try:
        test_conv_bn_act(act, use_res)
    finally:
        hip.HALO_FORCE = keep
    assert hip.HALO_COUNT[0] > before


@pytest.mark.parametrize("case,stages", [
    (c, st) for c in [CONV_CASES[i] for i in (0, 1, 3, 4, 5, 6, 7, 8, 12, 13, 14, 15)]
    for st in (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16)
    if _wgrad_stage_ok(c, st)])
def test_conv_wgrad_ring_variants(case, stages):
    """Weight-gradient kernel variants: 1-stage (occupancy), 2-stage ring, the 8-wave in-block
    2-way pixel split (stages=3), the 256x256 8-wave tile (stages=4, Cout >= 256), the 32-row tile
    (stages=5 / 6, Cout <= 32), the 4- / 3-deep rings of 32-pixel stages (stages=7 / 9 on the
    256x256 tile, 8 on the 4-wave tiles) and the prefetch-depth-2 kernel (csrc/wgrad_deep.hip, stages
    13 / 14 / 15: 256 x 256, 128 x 256, 256 x 128 on 4 waves, partial tiles included) - each over the
    tuner's split counts."""
    hip = _hip()
    keep, hip.WGRAD_STAGES = hip.WGRAD_STAGES, stages
    try:
        test_conv_fwd_bwd(case)
    finally:
        hip.WGRAD_STAGES = keep


@pytest.mark.parametrize("target", [8, 24, 48, 96, 192])
def test_wgrad_split_reduce_groups(target):
    """Split-K workspace reduce at every slab-group count (G = 1, 2, 4, 8, 16 for 8 / 24 / 48 / 96 / 192
    splits of a one-tile weight gradient): dW against the fp32 reference."""
    hip = _hip()
    keep = hip.WGRAD_TARGET_BLOCKS, hip.WGRAD_STAGES
    hip.WGRAD_TARGET_BLOCKS, hip.WGRAD_STAGES = target, 2
    try:
        test_conv_fwd_bwd((32, 64, 56, 56, 64, (1, 1), 1, (0, 0)))
    finally:
        hip.WGRAD_TARGET_BLOCKS, hip.WGRAD_STAGES = keep


@pytest.mark.parametrize("cfg", range(N_CFG))
@pytest.mark.parametrize("act,use_res", [("relu", True), ("silu", False)])
def test_conv_bn_act_tile_configs(act, use_res, cfg):
    """Fused epilogues (BN statistics, residual) on every configuration of the table."""
    hip = _hip()
    if cfg >= len(hip.conv_cfgs()):
        pytest.skip("past the configuration table")
    keep, hip.CONV_FORCE_CFG = hip.CONV_FORCE_CFG, (0, 0, cfg)
    try:
        test_conv_bn_act(act, use_res)
    finally:
        hip.CONV_FORCE_CFG = keep


@pytest.mark.parametrize("variant,single", [(1, 1), (2, 0), (2, 1000), (3, 1)])
@pytest.mark.parametrize("case", [CONV_CASES[1], CONV_CASES[3], CONV_CASES[7], CONV_CASES[10], CONV_CASES[12]])
def test_conv_kernel_variants(case, variant, single):
    """Every fwd/dgrad kernel variant (register-staged, LDS-DMA 1/2/3-stage ring) and both wgrad
    variants produce the same numbers as the fp32 reference.  ``single`` = largest k-step count
    that takes the 1-stage ring (0: never, 1000: always)."""
    hip = _hip()
    hip.C.conv_set_variant(variant)
    hip.C.conv_set_single_stage(single)
    hip.C.conv_set_wgrad_variant(1 if variant == 1 else 2)
    keep, hip.CONV_STAGES = hip.CONV_STAGES, "0"  # the k-step heuristic, not the per-shape tuner
    keep_w, hip.WGRAD_STAGES = hip.WGRAD_STAGES, (1 if single == 1000 else 2)
    try:
        test_conv_fwd_bwd(case)
    finally:
        hip.CONV_STAGES = keep
        hip.WGRAD_STAGES = keep_w
        hip.C.conv_set_variant(0)
        hip.C.conv_set_single_stage(4)
        hip.C.conv_set_wgrad_variant(0)


def test_stem_padded_input():
    """Cin=3 image -> prepare_input pads to 8 channels; weight padded inside the op."""
    hip = _hip()
    torch.manual_seed(1)
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(DEV).to(memory_format=CL)
    with torch.no_grad():
        conv.weight.copy_(bf(conv.weight))
    x = bf(torch.randn(2, 3, 32, 32, device=DEV))
    xp = hip.prepare_input(x)
    assert xp.shape[1] == 8
    y = hip.ConvFn.apply(xp, conv.weight, conv, False)
    yr = F.conv2d(x, conv.weight, None, 2, 3)
    assert rel_err(y, yr) < 1e-2
    g = bf(torch.randn_like(yr))
    y.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
    wr = torch.autograd.grad(F.conv2d(x, conv.weight, None, 2, 3), conv.weight, g)[0]
    assert rel_err(conv.weight.grad, wr) < 2e-2


@pytest.mark.parametrize("hw", [(64, 64), (224, 224), (36, 50)])
def test_stem_space_to_depth(hw):
    """7x7 stride-2 stem on the space-to-depth input (4x4 stride-1 conv over 16 channels): forward
    (conv -> BN -> ReLU), BN statistics and the weight gradient against fp32 torch."""
    hip = _hip()
    torch.manual_seed(5)
    h, w = hw
    conv = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(DEV).to(memory_format=CL)
    bn = nn.BatchNorm2d(64).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(bf(conv.weight))
    conv_r = nn.Conv2d(3, 64, 7, 2, 3, bias=False).to(DEV)
    bn_r = nn.BatchNorm2d(64).to(DEV)
    conv_r.load_state_dict(conv.state_dict())
    bn_r.load_state_dict(bn.state_dict())
    x = bf(torch.randn(2, 3, h, w, device=DEV))
    assert hip.stem_s2d_eligible(x, conv)
    assert hip.prepare_input(x, stem=conv) is x
    out = hip.conv_bn_act(x, conv, bn, "relu", None)
    yc = conv_r(x)
    ref = F.relu(bn_r(yc + (bf(yc) - yc).detach()))
    assert out.shape == ref.shape
    assert rel_err(out, ref) < 2e-2
    assert torch.allclose(bn.running_mean, bn_r.running_mean, rtol=1e-2, atol=1e-3)
    g = bf(torch.randn_like(ref))
    out.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
    ref.backward(g)
    assert rel_err(conv.weight.grad, conv_r.weight.grad) < 3e-2
    assert rel_err(bn.weight.grad, bn_r.weight.grad) < 3e-2


@pytest.mark.parametrize("hw", [(224, 224), (36, 50), (30, 18)])
def test_stem_direct_matches_gemm(hw):
    """The halo-tile stem kernel (csrc/stem.hip, partial edge tiles included) against the implicit-GEMM
    path on the same space-to-depth input: output and fused BN statistics."""
    hip = _hip()
    torch.manual_seed(6)
    h, w = hw
    n = 3
    x = torch.randn(n, 3, h, w, device=DEV)
    xs = hip._empty_cl(n, 16, h // 2, w // 2, DEV)
    hip.C.prepare_input_s2d(x, xs, n, h, w)
    g = hip._s2d_geom(n, h, w, 64)
    idx = hip._s2d_index(torch.device(DEV))  # KRSC position r*21 + s*3 + c -> s2d weight column
    wq = torch.zeros(64, 256, device=DEV)
    wq[:, idx] = torch.randn(64, 147, device=DEV) * 0.05  # taps outside the 7x7 window stay zero
    wq = wq.to(torch.bfloat16)
    m = g.N * g.OH * g.OW
    grp = hip.stat_groups(m)
    st_d = torch.zeros(grp * 2 * 64, device=DEV)
    y_d = hip._empty_cl(n, 64, g.OH, g.OW, DEV)
    hip.C.stem_conv(xs, wq.view(-1), y_d, st_d, grp, n, g.OH, g.OW)
    st_g = torch.zeros(grp * 2 * 64, device=DEV)
    y_g = hip.conv_forward_raw(xs, None, g, stats=st_g, wb=wq.view(-1))
    assert rel_err(y_d, y_g) < 1e-2
    sd, sg = st_d.view(grp, 2, 64).sum(0), st_g.view(grp, 2, 64).sum(0)
    assert rel_err(sd[0], sg[0]) < 1e-2 and rel_err(sd[1], sg[1]) < 1e-2
    # against fp32: the s2d conv equals the 7x7 stride-2 conv of the bf16-rounded image
    wr = wq.float()[:, idx].view(64, 7, 7, 3).permute(0, 3, 1, 2).contiguous()
    yr = F.conv2d(bf(x), wr, None, 2, 3)
    assert rel_err(y_d, yr) < 1e-2


@pytest.mark.parametrize("case", [
    # N, Cin, H, W, Cout, pad
    (2, 32, 37, 37, 32, 0),   # Inception Conv2d_2a (valid)
    (2, 32, 35, 35, 64, 1),   # Inception Conv2d_2b
    (2, 64, 56, 56, 64, 1),   # ResNet layer1
    (3, 64, 13, 70, 128, 1),  # two 64-channel output tiles, partial 8 x 32 tiles (variant 5)
    (1, 24, 19, 45, 40, 1),   # partial channel tiles, odd sizes
    (3, 8, 9, 17, 16, 0),
    (2, 80, 19, 19, 48, 0),   # Inception Conv2d_4a channels (96-padded variant)
])
def test_direct_conv(case):
    """Halo-tile direct 3x3 conv (csrc/direct_conv.hip), every variant that fits, against fp32 torch:
    output and fused BN statistics."""
    hip = _hip()
    n, cin, h, w, co, p = case
    torch.manual_seed(11)
    x = bf(torch.randn(n, cin, h, w, device=DEV))
    wt = bf(torch.randn(co, cin, 3, 3, device=DEV) * 0.1)
    yr = F.conv2d(x, wt, None, 1, p)
    oh, ow = yr.shape[2], yr.shape[3]
    xb = x.to(torch.bfloat16).contiguous(memory_format=CL)
    wk = wt.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    grp = hip.stat_groups(n * oh * ow)
    ran = 0
    for v, (cip, cot) in hip.DIRECT_CFGS.items():
        if cin > cip or (v == 5 and not (cin == 64 and (oh, ow) == (h, w))):
            continue
        y = hip._empty_cl(n, co, oh, ow, DEV)
        st = torch.zeros(grp * 2 * co, device=DEV)
        hip.C.direct_conv(xb, wk, y, st, grp, n, h, w, cin, oh, ow, co, p, p, v)
        assert rel_err(y, yr) < 1e-2, v
        sm = st.view(grp, 2, co).sum(0)
        yb = bf(yr)
        assert rel_err(sm[0], yb.sum((0, 2, 3))) < 1e-2, v
        assert rel_err(sm[1], (yb * yb).sum((0, 2, 3))) < 1e-2, v
        ran += 1
    assert ran > 0


def _direct_fits(case, variant):
    try:
        cip = _hip().DIRECT_CFGS[variant][0]
    except Exception:  # extension not importable: keep the case, the test skips it at run time
        return True
    return case[1] <= cip and case[3] <= cip


@pytest.mark.parametrize("case,variant", [
    (c, v) for c in [(2, 32, 23, 32, 0), (2, 32, 21, 64, 1), (2, 64, 20, 64, 1), (2, 80, 13, 80, 0)]
    for v in range(6) if _direct_fits(c, v)])
def test_direct_conv_chain(case, variant):
    """conv -> BN -> ReLU -> 3x3 conv -> BN with every eligible launch forced onto one direct-kernel
    variant: forward, and the second conv's data gradient with the fused BN-backward epilogue (the first
    BN's reduce) - against the GEMM configurations."""
    hip = _hip()
    n, c, hw, co, p = case
    cip, cot = hip.DIRECT_CFGS[variant]
    if c > cip or co > cip:
        pytest.skip("channels exceed the variant's padded input width")
    torch.manual_seed(12)
    mods = [nn.Conv2d(c, c, 3, 1, p, bias=False), nn.BatchNorm2d(c), nn.Conv2d(c, co, 3, 1, p, bias=False),
            nn.BatchNorm2d(co)]
    mods = [m.to(DEV).to(memory_format=CL) for m in mods]
    with torch.no_grad():
        for m in (mods[0], mods[2]):
            m.weight.copy_(bf(m.weight))
    x = bf(torch.randn(n, c, hw, hw, device=DEV))

    def run(force):
        keep, hip.DIRECT_FORCE = hip.DIRECT_FORCE, force
        keep_d, hip.DIRECT_CONV = hip.DIRECT_CONV, force is not None  # baseline: GEMM configurations only
        keep_g, hip.DIRECT_DGRAD = hip.DIRECT_DGRAD, True
        try:
            ms = [copy.deepcopy(m) for m in mods]
            xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
            a1 = hip.conv_bn_act(xb, ms[0], ms[1], "relu", None)
            out = hip.conv_bn_act(a1, ms[2], ms[3], None, None, exclusive_input=True)
            g = torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out).to(torch.bfloat16)
            out.backward(g.contiguous(memory_format=CL))
            return out.float(), xb.grad.float(), [p_.grad.float() for m in ms for p_ in m.parameters()]
        finally:
            hip.DIRECT_FORCE = keep
            hip.DIRECT_CONV = keep_d
            hip.DIRECT_DGRAD = keep_g

    o0, gx0, gp0 = run(None)
    o1, gx1, gp1 = run(variant)
    assert rel_err(o1, o0) < 2e-2
    assert rel_err(gx1, gx0) < 3e-2
    for a_, b_ in zip(gp1, gp0):
        assert rel_err(a_, b_) < 3e-2


def test_dense_conv_bn_act():
    """A conv whose kernel covers its whole input (Inception aux conv1, 5x5 on 5x5) runs as dense GEMMs:
    forward, BN statistics and every gradient against fp32 torch."""
    hip = _hip()
    torch.manual_seed(9)
    n, c, hw, co = 16, 128, 5, 96
    conv = nn.Conv2d(c, co, hw, bias=False).to(DEV).to(memory_format=CL)
    bn = nn.BatchNorm2d(co, eps=1e-3).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(bf(conv.weight))
    conv_r = nn.Conv2d(c, co, hw, bias=False).to(DEV)
    bn_r = nn.BatchNorm2d(co, eps=1e-3).to(DEV)
    conv_r.load_state_dict(conv.state_dict())
    bn_r.load_state_dict(bn.state_dict())
    x = bf(torch.randn(n, c, hw, hw, device=DEV))
    xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    assert hip.dense_conv_eligible(xb, conv)

    def no_library_gemm(*a, **k):
        raise AssertionError("dense conv must run on the in-tree MFMA kernels, not a library GEMM")
    keep_mm, keep_mat = torch.mm, torch.matmul
    torch.mm = torch.matmul = no_library_gemm
    try:
        out = hip.conv_bn_act(xb, conv, bn, "relu", None)
    finally:
        torch.mm, torch.matmul = keep_mm, keep_mat
    xr = x.clone().requires_grad_(True)
    yc = conv_r(xr)
    ref = F.relu(bn_r(yc + (bf(yc) - yc).detach()))
    assert out.shape == ref.shape == (n, co, 1, 1)
    assert rel_err(out, ref) < 2e-2
    assert torch.allclose(bn.running_mean, bn_r.running_mean, rtol=1e-2, atol=1e-3)
    g = bf(torch.randn_like(ref))
    torch.mm = torch.matmul = no_library_gemm
    try:
        out.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
    finally:
        torch.mm, torch.matmul = keep_mm, keep_mat
    ref.backward(g)
    assert rel_err(xb.grad, xr.grad) < 3e-2
    assert rel_err(conv.weight.grad, conv_r.weight.grad) < 3e-2
    assert rel_err(bn.weight.grad, bn_r.weight.grad) < 3e-2


def test_weight_shadow_follows_outside_writes():
    """The conv kernels read bf16 (and transposed / MX) shadows of the fp32 weights that the fused Adam
    keeps current.  A write to the weights outside the optimizer - load_state_dict between steps, an
    in-place edit - must reach the next forward and backward (ops/hip.py weight_bf16)."""
    from pytorch_imageclassification_distributed_amd.engine.optim import FusedAdam
    hip = _hip()
    torch.manual_seed(21)
    conv = nn.Conv2d(64, 64, 3, 1, 1, bias=False).to(DEV).to(memory_format=CL)
    bn = nn.BatchNorm2d(64).to(DEV)
    opt = FusedAdam(list(conv.parameters()) + list(bn.parameters()), lr=1e-3)
    x = bf(torch.randn(4, 64, 14, 14, device=DEV)).to(torch.bfloat16).contiguous(memory_format=CL)

    def step():
        xb = x.detach().clone().requires_grad_(True)
        out = hip.conv_bn_act(xb, conv, bn, "relu", None)
        opt.zero_grad(set_to_none=True)
        out.float().square().mean().backward()
        opt.step()
        return out.detach(), xb.grad.detach()

    step()
    step()  # the optimizer now owns the shadows (fused refresh)
    fresh = nn.Conv2d(64, 64, 3, 1, 1, bias=False).to(DEV).to(memory_format=CL)
    conv.load_state_dict(fresh.state_dict())  # an outside write between steps
    bn_ref = copy.deepcopy(bn)
    conv_ref = copy.deepcopy(conv)
    out, gx = step()
    xr = x.float().requires_grad_(True)
    yc = conv_ref(xr)
    ref = F.relu(bn_ref(yc + (bf(yc) - yc).detach()))
    ref.square().mean().backward()
    assert rel_err(out, ref) < 3e-2, "forward used a stale bf16 weight shadow"
    assert rel_err(gx, xr.grad) < 5e-2, "dgrad used a stale transposed weight shadow"
    with torch.no_grad():
        conv.weight.mul_(-1.0)  # in-place edit (after the optimizer step above): bumps the version counter
    conv_ref2 = copy.deepcopy(conv)
    xb = x.detach().clone()
    out2 = hip.conv_bn_act(xb, conv, copy.deepcopy(bn).eval(), None, None)
    ref2 = copy.deepcopy(bn).eval()(conv_ref2(x.float()))
    assert rel_err(out2, ref2) < 3e-2, "in-place weight edit not seen by the next forward"


@pytest.mark.parametrize("act,use_res", [("relu", False), ("relu", True), (None, False), ("silu", False)])
def test_conv_bn_act(act, use_res):
    hip = _hip()
    torch.manual_seed(2)
    n, c, h, w, co = 4, 64, 14, 14, 128
    conv = nn.Conv2d(c, co, 3, 1, 1, bias=False).to(DEV).to(memory_format=CL)
    bn = nn.BatchNorm2d(co).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(bf(conv.weight))
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv_r = nn.Conv2d(c, co, 3, 1, 1, bias=False).to(DEV)
    bn_r = nn.BatchNorm2d(co).to(DEV)
    conv_r.load_state_dict(conv.state_dict())
    bn_r.load_state_dict(bn.state_dict())
    x = bf(torch.randn(n, c, h, w, device=DEV))
    res = bf(torch.randn(n, co, h, w, device=DEV)) if use_res else None
    xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    rb = res.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True) if use_res else None
    out = hip.conv_bn_act(xb, conv, bn, act, rb)
    xr = x.clone().requires_grad_(True)
    rr = res.clone().requires_grad_(True) if use_res else None
    yc = conv_r(xr)
    yc = yc + (bf(yc) - yc).detach()  # the HIP path stores the conv output in bf16: same values here
    z = bn_r(yc)
    if use_res:
        z = z + rr
    ref = {None: z, "relu": F.relu(z) if act == "relu" else z, "silu": F.silu(z)}[act]
    assert rel_err(out, ref) < 2e-2
    assert torch.allclose(bn.running_mean, bn_r.running_mean, rtol=1e-2, atol=1e-3)
    assert torch.allclose(bn.running_var, bn_r.running_var, rtol=1e-2, atol=1e-3)
    assert int(bn.num_batches_tracked) == 1
    g = bf(torch.randn_like(ref))
    out.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
    ref.backward(g)
    assert rel_err(xb.grad, xr.grad) < 3e-2
    assert mean_err(xb.grad, xr.grad) < 1e-2
    assert rel_err(bn.weight.grad, bn_r.weight.grad) < 3e-2
    assert rel_err(bn.bias.grad, bn_r.bias.grad) < 3e-2
    assert rel_err(conv.weight.grad, conv_r.weight.grad) < 3e-2
    if use_res:
        assert rel_err(rb.grad, rr.grad) < 3e-2
    # eval mode uses running statistics
    bn.eval()
    bn_r.eval()
    with torch.no_grad():
        oe = hip.conv_bn_act(xb.detach(), conv, bn, act, rb.detach() if use_res else None)
        ze = bn_r(conv_r(x)) + (res if use_res else 0)
        re = {None: ze, "relu": F.relu(ze) if act == "relu" else ze, "silu": F.silu(ze)}[act]
    assert rel_err(oe, re) < 2e-2
    # eval-mode backward (frozen statistics: dy = scale * dz, no batch-statistics terms)
    for p_ in list(conv.parameters()) + list(bn.parameters()) + list(conv_r.parameters()) + list(bn_r.parameters()):
        p_.grad = None
    xe = xb.detach().clone().requires_grad_(True)
    oe = hip.conv_bn_act(xe, conv, bn, act, rb.detach() if use_res else None)
    xer = x.clone().requires_grad_(True)
    yce = conv_r(xer)
    ze = bn_r(yce + (bf(yce) - yce).detach()) + (res if use_res else 0)
    re = {None: ze, "relu": F.relu(ze) if act == "relu" else ze, "silu": F.silu(ze)}[act]
    ge = bf(torch.randn_like(re))
    oe.backward(ge.to(torch.bfloat16).contiguous(memory_format=CL))
    re.backward(ge)
    assert rel_err(xe.grad, xer.grad) < 3e-2
    assert rel_err(bn.weight.grad, bn_r.weight.grad) < 3e-2
    assert rel_err(bn.bias.grad, bn_r.bias.grad) < 3e-2
    assert rel_err(conv.weight.grad, conv_r.weight.grad) < 3e-2


def test_depthwise_bn_silu():
    hip = _hip()
    torch.manual_seed(3)
    # k3/k5 take the unrolled kernels (odd and even sizes, both strides); k7 the generic ones
    for (c, k, s, hw) in [(96, 3, 2, 28), (144, 5, 1, 14), (32, 3, 1, 16), (40, 5, 2, 15), (24, 3, 2, 9),
                          (16, 7, 1, 12), (48, 7, 2, 13)]:
        conv = nn.Conv2d(c, c, k, s, 0, groups=c, bias=False).to(DEV).to(memory_format=CL)
        conv.tf_same = True
        bn = nn.BatchNorm2d(c, eps=1e-3, momentum=0.01).to(DEV)
        with torch.no_grad():
            conv.weight.copy_(bf(conv.weight))
        x = bf(torch.randn(2, c, hw, hw, device=DEV))
        xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
        out = hip.conv_bn_act(xb, conv, bn, "silu", None)
        from pytorch_imageclassification_distributed_amd.ops.functional import conv_padding
        pt, pb, pl, pr = conv_padding(conv, hw, hw)
        xr = x.clone().requires_grad_(True)
        wr = conv.weight.detach().clone().requires_grad_(True)
        z = F.conv2d(F.pad(xr, (pl, pr, pt, pb)), wr, None, s, 0, 1, c)
        ref = F.silu(F.batch_norm(z, None, None, training=True, eps=1e-3))
        assert rel_err(out, ref) < 2e-2
        g = bf(torch.randn_like(ref))
        out.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
        ref.backward(g)
        assert rel_err(xb.grad, xr.grad) < 3e-2
        assert rel_err(conv.weight.grad, wr.grad) < 3e-2


@pytest.mark.parametrize("case", [
    # N, Cin, H, Cout, conv k/s/p, pool k/s/p
    (2, 3, 64, 64, (7, 2, 3), (3, 2, 1)),     # ResNet stem (space-to-depth conv path)
    (2, 32, 35, 64, (3, 1, 1), (3, 2, 0)),    # Inception Conv2d_2b -> maxpool (odd size, no padding)
    (1, 16, 17, 48, (3, 1, 0), (3, 2, 1)),
])
@pytest.mark.parametrize("stem_xa", [True, False])
def test_conv_bn_act_pool(case, stem_xa):
    """Stem fusion: max_pool2d(relu(bn(conv(x)))) - forward, running stats and every gradient, against
    the fp32 reference and (tightly) against the unfused HIP composition conv_bn_act -> max_pool2d.  With
    STEM_XA (ResNet stem) the pool backward masks by the pooled output and the stem conv's weight gradient
    forms dY itself from the BN's dz and map (no bn_bwd_elemt pass)."""
    import copy
    hip = _hip()
    keep_xa = hip.STEM_XA
    hip.STEM_XA = stem_xa
    try:
        _conv_bn_act_pool_case(hip, case, stem_xa)
    finally:
        hip.STEM_XA = keep_xa


def test_stem_xa_wgrad_64x256():
    """The s2d stem's XA weight gradient on the 64 x 256 tile (stages 16: Cout 64 x Ntot 256 in one column tile)."""
    hip = _hip()
    keep = hip.STEM_XA, hip.WGRAD_STAGES
    hip.STEM_XA, hip.WGRAD_STAGES = True, 16
    try:
        _conv_bn_act_pool_case(hip, (2, 3, 64, 64, (7, 2, 3), (3, 2, 1)), True)
    finally:
        hip.STEM_XA, hip.WGRAD_STAGES = keep


def _conv_bn_act_pool_case(hip, case, stem_xa):
    import copy
    n, cin, h, co, (k, s, p), pool = case
    torch.manual_seed(7)
    conv = nn.Conv2d(cin, co, k, s, p, bias=False).to(DEV).to(memory_format=CL)
    bn = nn.BatchNorm2d(co).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(bf(conv.weight))
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv_u, bn_u = copy.deepcopy(conv), copy.deepcopy(bn)
    conv_r = nn.Conv2d(cin, co, k, s, p, bias=False).to(DEV)
    bn_r = nn.BatchNorm2d(co).to(DEV)
    conv_r.load_state_dict(conv.state_dict())
    bn_r.load_state_dict(bn.state_dict())
    x = bf(torch.randn(n, cin, h, h, device=DEV))
    stem = cin == 3

    def inp():
        return x if stem else x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)

    xb, xu = inp(), inp()
    n_xa, n_red = hip.STEM_XA_COUNT[0], hip.POOL_BN_REDUCE_COUNT[0]
    out = hip.conv_bn_act_pool(xb, conv, bn, "relu", pool)
    unf = hip.max_pool2d(hip.conv_bn_act(xu, conv_u, bn_u, "relu", None), *pool)
    xr = x.clone().requires_grad_(not stem)
    yc = conv_r(xr)
    yc = yc + (bf(yc) - yc).detach()
    act = F.relu(bn_r(yc))
    # pooled at bf16, as the unfused bn_apply -> maxpool path stores the activation: bf16 ties pick the
    # same (first) window position in both
    ref = F.max_pool2d(act + (bf(act) - act).detach(), *pool)
    assert out.shape == ref.shape
    assert torch.equal(out, unf)
    assert rel_err(out, ref) < 2e-2
    assert torch.allclose(bn.running_mean, bn_r.running_mean, rtol=1e-2, atol=1e-3)
    assert torch.allclose(bn.running_var, bn_r.running_var, rtol=1e-2, atol=1e-3)
    g = bf(torch.randn_like(ref))
    gb = g.to(torch.bfloat16).contiguous(memory_format=CL)
    out.backward(gb)
    assert (hip.STEM_XA_COUNT[0] > n_xa) == (stem and stem_xa)
    # (the pool backward also took the BN-backward partial sums: no separate reduce pass)
    assert (hip.POOL_BN_REDUCE_COUNT[0] > n_red) == (stem and stem_xa and hip.POOL_BN_REDUCE)
    unf.backward(gb)
    ref.backward(g)
    # the fused gather matches the unfused maxpool_bwd -> BN backward (which rounds the full-resolution
    # gradient to bf16 in between)
    for a_, b_ in ((bn.weight.grad, bn_u.weight.grad), (bn.bias.grad, bn_u.bias.grad),
                   (conv.weight.grad, conv_u.weight.grad)) + (() if stem else ((xb.grad, xu.grad),)):
        assert rel_err(a_, b_) < 1e-2
    # vs fp32: a 1-ulp difference in the bf16 conv output can flip relu'(z) at |z| ~ 0 for a routed pixel;
    # the max-pool concentrates the gradient, so single elements move - compare mean errors
    for a_, b_ in ((bn.weight.grad, bn_r.weight.grad), (bn.bias.grad, bn_r.bias.grad),
                   (conv.weight.grad, conv_r.weight.grad)) + (() if stem else ((xb.grad, xr.grad),)):
        assert mean_err(a_, b_) < 6e-2  # (the unfused path, checked equal above, measures the same)
    bn.eval()
    bn_u.eval()
    with torch.no_grad():
        fused = hip.conv_bn_act_pool(xb.detach() if not stem else xb, conv, bn, "relu", pool)
        plain = hip.max_pool2d(hip.conv_bn_act(xb.detach() if not stem else xb, conv, bn, "relu", None), *pool)
    assert torch.equal(fused, plain)


@pytest.mark.parametrize("hw", [17, 16])
@pytest.mark.parametrize("kind", ["max311", "max320", "max321", "max220", "max120", "avg311", "avg530"])
def test_pools(kind, hw):
    """max320 / max321 / max220 / max120 take the stride-2 quad-gather backward, max311 the 2x2-candidate
    one; odd and even input sizes (the quad grid's last row / column is half outside the input on one)."""
    hip = _hip()
    torch.manual_seed(4)
    x = bf(torch.randn(2, 64, hw, hw + 1, device=DEV))
    xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    k, s, p = int(kind[3]), int(kind[4]), int(kind[5])
    if kind.startswith("max"):
        y, yr = hip.max_pool2d(xb, k, s, p), F.max_pool2d(xr, k, s, p)
    else:
        y, yr = hip.avg_pool2d(xb, k, s, p), F.avg_pool2d(xr, k, s, p)
    assert rel_err(y, yr) < 1e-2
    g = bf(torch.randn_like(yr))
    y.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
    yr.backward(g)
    assert rel_err(xb.grad, xr.grad) < 2e-2


@pytest.mark.parametrize("which", ["pools", "depthwise", "se", "stem_pool", "gap"])
def test_div64_fallback_paths(which):
    """The 64-bit index decode (taken above 2^31 work items, never at test sizes) forced on by the
    set_force_div64 hook: the same numerics tests must pass on that branch."""
    hip = _hip()
    hip.set_force_div64(True)
    try:
        if which == "pools":
            for kind in ("max311", "max320", "max321", "avg311", "avg530"):
                for hw in (16, 17):
                    test_pools(kind, hw)
        elif which == "depthwise":
            test_depthwise_bn_silu()
        elif which == "se":
            test_se_gate_and_misc()
        elif which == "stem_pool":
            # (the ReLU-masked pool backward of STEM_XA is a quad-kernel form, which the forced decode turns off)
            test_conv_bn_act_pool((2, 3, 64, 64, (7, 2, 3), (3, 2, 1)), False)
            test_conv_bn_act_pool((2, 32, 35, 64, (3, 1, 1), (3, 2, 0)), False)
        else:
            test_gap_head_ce()
    finally:
        hip.set_force_div64(False)


def test_gap_head_ce():
    hip = _hip()
    from pytorch_imageclassification_distributed_amd.models import mlp_head
    torch.manual_seed(5)
    x = bf(torch.randn(8, 256, 7, 7, device=DEV))
    xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    head = mlp_head(256, 7).to(DEV)
    w = torch.tensor([3, 3, 10, 1, 4, 4, 5], dtype=torch.float32, device=DEV)
    lab = torch.randint(0, 7, (8,), device=DEV)
    loss = hip.cross_entropy(hip.mlp(hip.global_avg_pool(xb), head), lab, w)
    head_r = mlp_head(256, 7).to(DEV)
    head_r.load_state_dict(head.state_dict())
    xr = x.clone().requires_grad_(True)
    loss_r = F.cross_entropy(head_r(F.adaptive_avg_pool2d(xr, 1).flatten(1)), lab, weight=w)
    assert abs(loss.item() - loss_r.item()) < 1e-4 * max(1.0, abs(loss_r.item()))
    (0.7 * loss).backward()
    (0.7 * loss_r).backward()
    assert rel_err(xb.grad, xr.grad) < 1e-2
    for (n1, p1), (_n2, p2) in zip(head.named_parameters(), head_r.named_parameters()):
        assert rel_err(p1.grad, p2.grad) < 1e-4, n1


def test_se_gate_and_misc():
    hip = _hip()
    torch.manual_seed(6)
    c, nsq = 96, 4
    red = nn.Conv2d(c, nsq, 1).to(DEV)
    exp = nn.Conv2d(nsq, c, 1).to(DEV)
    x = bf(torch.randn(2, c, 9, 9, device=DEV))
    xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    y = hip.se_gate(xb, red, exp)
    xr = x.clone().requires_grad_(True)
    pool = xr.mean((2, 3))
    hid = F.silu(F.linear(pool, red.weight.flatten(1), red.bias))
    s = torch.sigmoid(F.linear(hid, exp.weight.flatten(1), exp.bias))[:, :, None, None]
    yr = s * xr
    assert rel_err(y, yr) < 1e-2
    g = bf(torch.randn_like(yr))
    y.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
    gr = torch.autograd.grad(yr, [xr, red.weight, exp.weight], g)
    assert rel_err(xb.grad, gr[0]) < 2e-2
    # cat / add
    a = torch.randn(2, 16, 5, 5, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    b = torch.randn(2, 24, 5, 5, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    assert torch.equal(hip.cat_channels([a, b]), torch.cat([a, b], 1))
    assert rel_err(hip.add(a, a), a.float() * 2) < 1e-2


def test_fused_adam_matches_torch():
    from pytorch_imageclassification_distributed_amd.engine.optim import FusedAdam
    torch.manual_seed(7)
    p1 = torch.randn(4097, device=DEV, requires_grad=True)
    p2 = torch.randn(64, 3, 3, 3, device=DEV).contiguous(memory_format=CL).requires_grad_(True)
    q1, q2 = p1.detach().clone().requires_grad_(True), p2.detach().clone().requires_grad_(True)
    opt = FusedAdam([p1, p2], lr=1e-2)
    ref = torch.optim.Adam([q1, q2], lr=1e-2)
    for _ in range(5):
        g1, g2 = torch.randn_like(p1), torch.randn_like(p2)
        p1.grad, p2.grad = g1.clone(), g2.clone().contiguous(memory_format=CL)
        q1.grad, q2.grad = g1.clone(), g2.clone()
        opt.step()
        ref.step()
    assert torch.allclose(p1, q1, atol=1e-5, rtol=1e-5)
    assert torch.allclose(p2, q2, atol=1e-5, rtol=1e-5)
    sd = opt.state_dict()
    assert float(sd["state"][0]["step"]) == 5.0


def test_adam_maintains_weight_shadows():
    """After fused-Adam steps the bf16 KRSC shadow and the transposed [Ci][T][Co] dgrad shadow
    (rewritten inside the Adam kernel, never re-transposed) equal a fresh cast of the weights."""
    from pytorch_imageclassification_distributed_amd.engine.optim import FusedAdam
    hip = _hip()
    torch.manual_seed(9)
    conv = nn.Conv2d(32, 48, 3, 1, 1, bias=False).to(DEV).to(memory_format=CL)
    dw = nn.Conv2d(48, 48, 5, 1, 2, groups=48, bias=False).to(DEV).to(memory_format=CL)
    opt = FusedAdam(list(conv.parameters()) + list(dw.parameters()), lr=1e-2)
    x = torch.randn(2, 32, 12, 12, device=DEV).to(torch.bfloat16).contiguous(memory_format=CL)
    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        xx = x.clone().requires_grad_(True)
        y = hip.ConvFn.apply(xx, conv.weight, conv, False)
        z = hip.DwConvFn.apply(y, dw.weight, dw)
        z.float().square().mean().backward()
        opt.step()
    torch.cuda.synchronize()
    for w, ci in ((conv.weight, 32), (dw.weight, 1)):
        co, t = w.shape[0], w.shape[2] * w.shape[3]
        e = hip._SHADOWS[id(w)]
        assert e.fused and e.tfused
        krsc = w.detach().permute(0, 2, 3, 1).reshape(co, t, ci).to(torch.bfloat16)
        assert torch.equal(hip.weight_bf16(w).view(co, t, ci), krsc)
        assert torch.equal(hip.weight_bf16_t(w, co, t, ci).view(ci, t, co), krsc.permute(2, 1, 0))


def test_resnet18_matches_reference_path():
    """Whole-model forward/backward: HIP bf16 path vs ATen fp32 path on identical weights.

    Gradient agreement is measured by cosine similarity per layer and compared with what
    the reference stack itself achieves in bf16 autocast (same weights, same data): the
    HIP path must be at least as close to fp32 as torch's own bf16 path, minus a margin.
    """
    from pytorch_imageclassification_distributed_amd.models import Classifier
    from pytorch_imageclassification_distributed_amd.ops import functional as Fx
    torch.manual_seed(8)
    base = Classifier("resnet18", 7)
    with torch.no_grad():
        for p in base.parameters():
            p.copy_(bf(p))
    sd = base.state_dict()
    x = bf(torch.randn(16, 3, 64, 64, device=DEV))
    lab = torch.randint(0, 7, (16,), device=DEV)
    layers = ["encoder.fc.6.weight", "encoder.layer4.1.conv2.weight", "encoder.layer3.0.conv1.weight",
              "encoder.layer2.0.conv1.weight", "encoder.layer1.0.conv1.weight", "encoder.conv1.weight"]

    def run(backend, autocast):
        m = Classifier("resnet18", 7).to(DEV)
        m.load_state_dict(sd)
        if backend == "hip":
            m = m.to(memory_format=CL)
        Fx.set_backend(backend)
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
                out = m(x)
            loss = Fx.cross_entropy(out.float(), lab)
            loss.backward()
        finally:
            Fx.set_backend("auto")
        g = dict(m.named_parameters())
        return loss.item(), {k: g[k].grad.float().flatten() for k in layers}

    l32, g32 = run("torch", False)
    lbf, gbf = run("torch", True)
    lh, gh = run("hip", False)
    assert abs(lh - l32) < 0.02 * abs(l32) + 1e-3
    for k in layers:
        c_h = F.cosine_similarity(gh[k], g32[k], dim=0).item()
        c_t = F.cosine_similarity(gbf[k], g32[k], dim=0).item()
        print(f"{k}: cos(hip, fp32)={c_h:.4f} cos(torch-bf16, fp32)={c_t:.4f}")
        assert c_h > min(0.98, c_t - 0.05), (k, c_h, c_t)


def test_grad_slot_fused_accumulation():
    """Block input feeding two convs: the slot-fused dgrad (epilogue addend) equals autograd's sum."""
    hip = _hip()
    torch.manual_seed(9)
    c1 = nn.Conv2d(64, 32, 1, bias=False).to(DEV).to(memory_format=CL)
    c2 = nn.Conv2d(64, 128, 1, 2, bias=False).to(DEV).to(memory_format=CL)
    x = torch.randn(2, 64, 14, 14, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    xa = x.clone().requires_grad_(True)
    slot = hip.GradSlot()
    ya = hip.ConvFn.apply(xa, c1.weight, c1, False, slot)
    za = hip.ConvFn.apply(xa, c2.weight, c2, False, slot)
    (ya.float().square().sum() + za.float().sum()).backward()
    xb = x.clone().requires_grad_(True)
    yb = hip.ConvFn.apply(xb, c1.weight, c1, False)
    zb = hip.ConvFn.apply(xb, c2.weight, c2, False)
    (yb.float().square().sum() + zb.float().sum()).backward()
    assert slot.t is None
    assert rel_err(xa.grad, xb.grad) < 1e-2


def _mx_dequant(q, sc, shape):
    """fp8 e4m3 bytes + E8M0 per-32 scales -> fp32 (torch reference decode)."""
    v = q.view(torch.float8_e4m3fn).float().reshape(-1, 32)
    s = torch.exp2(sc.float() - 127.0).reshape(-1, 1)
    return (v * s).reshape(shape)


def test_mx_quant_activation():
    """bf16 -> MX-FP8: block scale = smallest power of two putting the block max <= 448, elements
    rounded to nearest e4m3 (identical bytes to torch's float8_e4m3fn cast of the scaled block)."""
    hip = _hip()
    torch.manual_seed(11)
    x = (torch.randn(6, 256, 7, 5, device=DEV) * torch.logspace(-3, 3, 256, device=DEV).view(1, -1, 1, 1))
    xb = x.to(torch.bfloat16).contiguous(memory_format=CL)
    q, sc = hip.act_mx(xb)
    flat = xb.permute(0, 2, 3, 1).reshape(-1, 32).float()
    amax = flat.abs().amax(1)
    e = torch.ceil(torch.log2(amax / 448.0)).clamp(-127, 127)
    assert torch.equal(sc.long(), (e + 127).long())
    ref = (flat * torch.exp2(-e).unsqueeze(1)).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert torch.equal(q.view(torch.uint8), ref.view(torch.uint8).reshape(-1))
    deq = _mx_dequant(q, sc, flat.shape)
    assert ((deq - flat).abs() <= flat.abs() * 2 ** -3 + amax.unsqueeze(1) * 2 ** -9).all()


@pytest.mark.parametrize("shape", [(256, 128, 1, 1, 14), (128, 256, 3, 1, 12), (256, 256, 3, 2, 13), (512, 64, 1, 1, 7),
                                   (256, 512, 1, 2, 14)])
def test_fp8_conv_forward(shape):
    """MX-FP8 forward conv (v_mfma_scale_f32_16x16x128_f8f6f4) == fp32 conv of the dequantised
    operands (exact products, fp32 accumulation), and within fp8 quantisation error of the bf16 conv."""
    hip = _hip()
    ci, co, k, s, hw = shape
    torch.manual_seed(12)
    conv = nn.Conv2d(ci, co, k, s, k // 2, bias=False).to(DEV).to(memory_format=CL)
    x = torch.randn(3, ci, hw, hw, device=DEV).to(torch.bfloat16).contiguous(memory_format=CL)
    y16 = hip.ConvFn.apply(x, conv.weight, conv, False)
    hip.set_fp8(True)
    try:
        y8 = hip.ConvFn.apply(x, conv.weight, conv, True)  # with the fused BN-statistics epilogue
        part = hip.ws(x.device).stats_buf(co)
        sums = torch.empty(2 * co, dtype=torch.float64, device=DEV)
        hip.C.bn_partials(part, hip.G_STATS, co, sums, None, None)  # consume (and re-zero) the partials
        yf = y8.float().permute(0, 2, 3, 1).reshape(-1, co)
        torch.testing.assert_close(sums[:co].float(), yf.sum(0), rtol=1e-3, atol=1e-2)
        xq, xs = hip.act_mx(x)
        wq, wsc = hip.weight_mx(conv.weight)
    finally:
        hip.set_fp8(False)
    xd = _mx_dequant(xq, xs, (3, hw, hw, ci)).permute(0, 3, 1, 2)
    wd = _mx_dequant(wq, wsc, (co, k, k, ci)).permute(0, 3, 1, 2)
    ref = F.conv2d(xd, wd, None, s, k // 2)
    assert rel_err(y8, ref) < 1e-2
    assert rel_err(y8, y16.float()) < 8e-2


@pytest.mark.parametrize("cfg", range(N_FP8_CFG))
@pytest.mark.parametrize("shape", [(256, 128, 1, 1, 14), (128, 256, 3, 1, 12), (256, 512, 1, 2, 14)])
def test_fp8_conv_tile_configs(shape, cfg):
    """Every entry of the MX-FP8 kernel's configuration table (incl. the 256x256 8-wave tile)."""
    hip = _hip()
    if cfg >= len(hip.conv_fp8_cfgs()):
        pytest.skip("past the configuration table")
    keep, hip.CONV_FORCE_FP8_CFG = hip.CONV_FORCE_FP8_CFG, (0, 0, cfg)
    try:
        test_fp8_conv_forward(shape)
    finally:
        hip.CONV_FORCE_FP8_CFG = keep


def test_fp8_resnet50_step():
    """--dtype fp8 end to end on ResNet-50.  Train-mode gradients at random init are chaotic (BN
    gradient explosion amplifies any perturbation), so the checks are the well-posed ones: the
    eval-mode network (a fixed function) agrees with the bf16 path, and fp8 training steps on a fixed
    batch drive the loss down like bf16 does."""
    from pytorch_imageclassification_distributed_amd.engine.optim import FusedAdam
    from pytorch_imageclassification_distributed_amd.models import Classifier
    from pytorch_imageclassification_distributed_amd.ops import functional as Fx
    hip = _hip()
    torch.manual_seed(13)
    m = Classifier("resnet50", 7).to(DEV).to(memory_format=CL)
    x = torch.randn(16, 3, 96, 96, device=DEV)
    y = torch.randint(0, 7, (16,), device=DEV)
    m.eval()
    with torch.no_grad():
        l16 = m(x).float()
        hip.set_fp8(True)
        try:
            l8 = m(x).float()
        finally:
            hip.set_fp8(False)
    assert torch.nn.functional.cosine_similarity(l16.flatten(), l8.flatten(), 0).item() > 0.98
    m.train()
    opt = FusedAdam(m.parameters(), lr=1e-3)
    losses = []
    hip.set_fp8(True)
    try:
        for _ in range(8):
            opt.zero_grad(set_to_none=True)
            loss = Fx.cross_entropy(m(x), y)
            loss.backward()
            opt.step()  # also refreshes the MX weight copies
            losses.append(loss.item())
    finally:
        hip.set_fp8(False)
    assert all(math.isfinite(v) for v in losses)
    assert losses[-1] < 0.7 * losses[0], losses


def test_bn_apply_emits_mx_copy():
    """In fp8 mode BN-apply writes the MX-FP8 copy of its output itself (no separate quantisation
    pass); it is attached to the returned activation and byte-identical to quantising that output."""
    hip = _hip()
    torch.manual_seed(14)
    conv = nn.Conv2d(128, 256, 1, bias=False).to(DEV).to(memory_format=CL)
    bn = nn.BatchNorm2d(256).to(DEV)
    x = torch.randn(4, 128, 9, 9, device=DEV).to(torch.bfloat16).contiguous(memory_format=CL)
    hip.set_fp8(True)
    try:
        out = hip.conv_bn_act(x, conv, bn, "relu", None)
        mx = getattr(out, "_imgcls_mx", None)
        assert mx is not None and mx[2] == out._version
        q, qs = mx[0].clone(), mx[1].clone()
        del out._imgcls_mx
        q2, qs2 = hip.act_mx(out)
    finally:
        hip.set_fp8(False)
    assert torch.equal(qs, qs2)
    assert torch.equal(q.view(torch.uint8), q2.view(torch.uint8))



@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("n,c,nsq,hw", [(2, 96, 4, 9), (40, 144, 6, 7), (3, 1152, 48, 5), (33, 240, 10, 4),
                                        (5, 2560, 160, 2), (300, 96, 4, 3), (1024, 240, 10, 2)])
def test_se_gate_fused_grads(n, c, nsq, hw, fused):
    """SE MLP (csrc/se.hip fused kernels and the GEMM/activation fallback) against fp32 autograd: output,
    input gradient and all four weight / bias gradients; batches above the 32-image LDS chunk and hidden
    sizes that are not multiples of 4; batches of 300 / 1024 split the weight gradients into 3 / 8 slices."""
    hip = _hip()
    torch.manual_seed(n * 7 + c)
    red = nn.Conv2d(c, nsq, 1).to(DEV)
    exp = nn.Conv2d(nsq, c, 1).to(DEV)
    x = bf(torch.randn(n, c, hw, hw, device=DEV))
    xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    keep = hip.SE_FUSED
    hip.SE_FUSED = fused
    try:
        y = hip.se_gate(xb, red, exp)
        g = bf(torch.randn_like(y.float()))
        y.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
        torch.cuda.synchronize()
    finally:
        hip.SE_FUSED = keep
    xr = x.clone().requires_grad_(True)
    wr = red.weight.detach().clone().requires_grad_(True)
    br = red.bias.detach().clone().requires_grad_(True)
    we = exp.weight.detach().clone().requires_grad_(True)
    be = exp.bias.detach().clone().requires_grad_(True)
    hid = F.silu(F.linear(xr.mean((2, 3)), wr.flatten(1), br))
    yr = torch.sigmoid(F.linear(hid, we.flatten(1), be))[:, :, None, None] * xr
    yr.backward(g)
    assert rel_err(y, yr) < 1e-2
    assert rel_err(xb.grad, xr.grad) < 2e-2
    for mine, ref in ((red.weight.grad, wr.grad), (red.bias.grad, br.grad), (exp.weight.grad, we.grad),
                      (exp.bias.grad, be.grad)):
        assert rel_err(mine.reshape(ref.shape), ref) < 2e-2


@pytest.mark.parametrize("per_image", [True, False])
@pytest.mark.parametrize("n,c,hw", [(4, 96, 14), (3, 1152, 7), (2, 2064, 5), (2, 40, 57)])
def test_se_gate_fused_bn_backward(n, c, hw, per_image):
    """BN -> SiLU -> SE gate (exclusive consumer): se_dx emits dz and the BN's backward partial sums (BwdLink),
    with the per-image kernel (default) and the grid-stride one; gradients of the input and of every parameter
    match fp32 autograd."""
    hip = _hip()
    hip.C.se_set_dx_n(per_image)
    try:
        _se_gate_fused_case(hip, n, c, hw)
    finally:
        hip.C.se_set_dx_n(True)


def _se_gate_fused_case(hip, n, c, hw):
    torch.manual_seed(c)
    nsq = max(1, c // 24)
    conv = nn.Conv2d(c, c, 1, bias=False).to(DEV).to(memory_format=CL)
    bn = nn.BatchNorm2d(c, eps=1e-3).to(DEV)
    red = nn.Conv2d(c, nsq, 1).to(DEV)
    exp = nn.Conv2d(nsq, c, 1).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(bf(conv.weight))
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x = bf(torch.randn(n, c, hw, hw, device=DEV))
    xb = x.to(torch.bfloat16).contiguous(memory_format=CL).requires_grad_(True)
    before = hip.FUSED_BWD_COUNT[0]
    a = hip.conv_bn_act(xb, conv, bn, "silu", None)
    y = hip.se_gate(a, red, exp, exclusive_input=True)
    g = bf(torch.randn(y.shape, device=DEV))
    y.backward(g.to(torch.bfloat16).contiguous(memory_format=CL))
    torch.cuda.synchronize()
    assert hip.FUSED_BWD_COUNT[0] > before
    xr = x.clone().requires_grad_(True)
    ps = [p_.detach().clone().requires_grad_(True) for m in (conv, bn, red, exp) for p_ in m.parameters()]
    z = F.batch_norm(F.conv2d(xr, ps[0]), None, None, ps[1], ps[2], training=True, eps=1e-3)
    ar = F.silu(z)
    hid = F.silu(F.linear(ar.mean((2, 3)), ps[3].flatten(1), ps[4]))
    yr = torch.sigmoid(F.linear(hid, ps[5].flatten(1), ps[6]))[:, :, None, None] * ar
    yr.backward(g)
    assert rel_err(y, yr) < 2e-2
    assert rel_err(xb.grad, xr.grad) < 3e-2
    mine = [p_.grad for m in (conv, bn, red, exp) for p_ in m.parameters()]
    for i, (m_, r_) in enumerate(zip(mine, ps)):
        assert rel_err(m_.reshape(r_.grad.shape), r_.grad) < 3e-2, i


# ---------------------------------------------------------------------------------------------------------
# BN-backward elementwise fused into the producer 1x1 conv's dgrad / wgrad (ops/hip.py XaLink, csrc XA)
# ---------------------------------------------------------------------------------------------------------
def _xa_block(hip, n, cin, hw, cmid, stride, act, use_res, xa_on, cfg=None, wstages=None, k=1, xa_out=False):
    """x -> kxk conv (stride) -> BN -> act [+ res] -> 1x1 conv -> BN: the first BN's backward is linked to
    the second conv's dgrad (dz arrives fused), then handed to the first conv (XA).  Returns outputs and
    gradients, and how many BN backwards took the fused path."""
    torch.manual_seed(31)
    c1 = nn.Conv2d(cin, cmid, k, stride, k // 2, bias=False).to(DEV).to(memory_format=CL)
    b1 = nn.BatchNorm2d(cmid).to(DEV)
    c2 = nn.Conv2d(cmid, 256, 1, 1, 0, bias=False).to(DEV).to(memory_format=CL)
    b2 = nn.BatchNorm2d(256).to(DEV)
    with torch.no_grad():
        for m in (c1, c2):
            m.weight.copy_(bf(m.weight))
        b1.weight.uniform_(0.5, 1.5)
        b1.bias.uniform_(-0.5, 0.5)
    x = bf(torch.randn(n, cin, hw, hw, device=DEV)).to(torch.bfloat16).contiguous(memory_format=CL)
    oh = (hw + 2 * (k // 2) - k) // stride + 1
    res = bf(torch.randn(n, cmid, oh, oh, device=DEV)).to(torch.bfloat16).contiguous(memory_format=CL)
    keep = hip.FUSE_XA, hip.CONV_FORCE_CFG, hip.WGRAD_STAGES, hip.XA_MAX_REP, hip.XA_OUT
    hip.FUSE_XA, hip.XA_MAX_REP = xa_on, 10 ** 6  # every eligible geometry, whatever the cost gate says
    hip.XA_OUT = xa_out
    if cfg is not None:
        hip.CONV_FORCE_CFG = (0, 0, cfg)
    if wstages is not None:
        hip.WGRAD_STAGES = wstages
    n0 = hip.XA_COUNT[0]
    try:
        xb = x.detach().clone().requires_grad_(True)
        rb = res.detach().clone().requires_grad_(True) if use_res else None
        h = hip.conv_bn_act(xb, c1, b1, act, rb)
        out = hip.conv_bn_act(h, c2, b2, "relu", None, exclusive_input=True)
        g = torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out).to(torch.bfloat16)
        out.backward(g.contiguous(memory_format=CL))
        torch.cuda.synchronize()
        grads = [xb.grad.float(), c1.weight.grad.float(), b1.weight.grad.float(), b1.bias.grad.float(),
                 c2.weight.grad.float()] + ([rb.grad.float()] if use_res else [])
        return out.float(), grads, hip.XA_COUNT[0] - n0
    finally:
        hip.FUSE_XA, hip.CONV_FORCE_CFG, hip.WGRAD_STAGES, hip.XA_MAX_REP, hip.XA_OUT = keep


@pytest.mark.parametrize("case", [
    # n, cin, hw, cmid, stride, act, residual, kernel
    (4, 64, 28, 256, 1, "relu", True, 1),    # bn3-like: wide output, residual + ReLU
    (4, 256, 28, 64, 1, "relu", False, 1),   # bn1-like: narrow output
    (4, 128, 28, 128, 2, None, False, 1),    # downsample-like: stride 2, no activation
    (2, 512, 7, 512, 1, "relu", True, 1),    # 7x7 map, partial row tiles
    (3, 64, 15, 192, 1, "silu", False, 1),   # odd pixel count, SiLU
    (4, 64, 14, 64, 1, "relu", False, 3),    # bn2-like: 3x3 dgrad, padded taps masked
    (4, 128, 15, 128, 2, "relu", False, 3),  # 3x3 stride 2: sub-pixel phases, odd input
    # 64 input channels: the one-pass fused dgrad + wgrad kernel (conv_fused_bwd2 for 128 / 192 / 256 outputs) on
    # maps large enough that every persistent block walks several tiles (X slots alternate, epilogues in them)
    (8, 64, 112, 128, 1, "relu", False, 1),
    (8, 64, 112, 192, 1, "relu", True, 1),
    (6, 64, 113, 256, 1, None, True, 1),
])
def test_bn_backward_fused_into_producer_conv(case):
    """dgrad / wgrad with the fused BN-backward operand map against the unfused path (bn_bwd_elemt + plain
    GEMMs): same outputs, same gradients to bf16 accuracy, and the fused path really taken."""
    hip = _hip()
    n, cin, hw, cmid, stride, act, use_res, k = case
    o0, g0, k0 = _xa_block(hip, n, cin, hw, cmid, stride, act, use_res, False, k=k)
    o1, g1, k1 = _xa_block(hip, n, cin, hw, cmid, stride, act, use_res, True, k=k)
    assert k0 == 0 and k1 >= 1, (k0, k1)
    # (the forward is the same code both times; on maps of many blocks its BN statistics are summed by fp32
    # atomics in arrival order, so the two forwards agree to rounding, not bitwise)
    assert rel_err(o1, o0) < 1e-2 and mean_err(o1, o0) < 1e-3
    # the gradients inherit that forward rounding: on the 64-channel maps of 50 K+ pixels the BN-parameter
    # gradients (sums over every pixel of a bf16 dz) measured mean errors of 3-5.5e-3 from run to run
    mtol = 1e-2 if n * hw * hw > 50000 else 5e-3
    for a_, b_ in zip(g1, g0):
        assert rel_err(a_, b_) < 2e-2, rel_err(a_, b_)
        assert mean_err(a_, b_) < mtol, mean_err(a_, b_)


@pytest.mark.parametrize("case", [
    (4, 64, 28, 256, 1, "relu", True),     # bn3-like: wide output, residual + ReLU
    (4, 256, 28, 64, 1, "relu", False),    # bn1-like: narrow output, 4 dgrad column tiles (only tile 0 stores)
    (4, 128, 28, 128, 2, None, False),     # stride 2: dY stored from the single non-empty phase
    (2, 512, 7, 512, 1, "relu", True),     # partial row tiles
    (3, 64, 15, 192, 1, "silu", False),    # odd pixel count
])
def test_bn_backward_fused_dy_written_once(case):
    """XA_OUT: the data gradient stores the dY it forms (first column tile) and the weight gradient reads it
    plainly - same outputs and gradients as the in-kernel transform in both GEMMs and as the unfused path."""
    hip = _hip()
    n0 = hip.XA_OUT_COUNT[0]
    o0, g0, _ = _xa_block(hip, *case, xa_on=False)
    o1, g1, k1 = _xa_block(hip, *case, xa_on=True, xa_out=True)
    assert k1 >= 1 and hip.XA_OUT_COUNT[0] > n0
    assert torch.equal(o0, o1)
    for a_, b_ in zip(g1, g0):
        assert rel_err(a_, b_) < 2e-2, rel_err(a_, b_)
        assert mean_err(a_, b_) < 5e-3, mean_err(a_, b_)


def test_bn_backward_fused_every_kernel_variant():
    """Every conv configuration with a fused A-operand variant and every wgrad ring / tile variant with a
    fused dY form, on one bn3-like block, against the unfused path."""
    hip = _hip()
    case = (2, 64, 20, 256, 1, "relu", True)
    _o, g0, _ = _xa_block(hip, *case, xa_on=False)
    ran = 0
    for i in range(len(hip.conv_cfgs())):
        if not hip.C.conv_cfg_has_xa(i):
            continue
        for wst in (1, 2, 3, 4):
            _o, g1, k1 = _xa_block(hip, *case, xa_on=True, cfg=i, wstages=wst)
            assert k1 >= 1
            for a_, b_ in zip(g1, g0):
                assert rel_err(a_, b_) < 2e-2, (i, wst, rel_err(a_, b_))
            ran += 1
    assert ran >= 8


def _xf_block(hip, n, cin, hw, cmid, k, stride, act, xf_on, cout=128, cfg=None, wstages=None):
    """x -> 1x1 conv -> BN -> act (deferred: defer_act) -> kxk conv (stride) -> BN -> ReLU.  With XF the
    second conv applies the first BN on its operand loads (forward and weight gradient) and act(bn(y)) is
    never written.  Returns the output, the gradients and how many convs read a deferred BN output."""
    torch.manual_seed(37)
    c1 = nn.Conv2d(cin, cmid, 1, 1, 0, bias=False).to(DEV).to(memory_format=CL)
    b1 = nn.BatchNorm2d(cmid).to(DEV)
    c2 = nn.Conv2d(cmid, cout, k, stride, k // 2, bias=False).to(DEV).to(memory_format=CL)
    b2 = nn.BatchNorm2d(cout).to(DEV)
    with torch.no_grad():
        for m in (c1, c2):
            m.weight.copy_(bf(m.weight))
        b1.weight.uniform_(0.5, 1.5)
        b1.bias.uniform_(-0.5, 0.5)
    x = bf(torch.randn(n, cin, hw, hw, device=DEV)).to(torch.bfloat16).contiguous(memory_format=CL)
    keep = hip.FUSE_XF, hip.CONV_FORCE_CFG, hip.WGRAD_STAGES, hip.XF_MAX_REP
    hip.FUSE_XF, hip.XF_MAX_REP = xf_on, 10 ** 6
    if cfg is not None:
        hip.CONV_FORCE_CFG = (0, 0, cfg)
    if wstages is not None:
        hip.WGRAD_STAGES = wstages
    n0 = hip.XF_COUNT[0]
    try:
        xb = x.detach().clone().requires_grad_(True)
        h = hip.conv_bn_act(xb, c1, b1, act, None, defer_act=True)
        assert (getattr(h, "_imgcls_xf", None) is not None) == xf_on
        out = hip.conv_bn_act(h, c2, b2, "relu", None, exclusive_input=True)
        g = torch.linspace(-1, 1, out.numel(), device=DEV).view_as(out).to(torch.bfloat16)
        out.backward(g.contiguous(memory_format=CL))
        torch.cuda.synchronize()
        grads = [xb.grad.float(), c1.weight.grad.float(), b1.weight.grad.float(), b1.bias.grad.float(),
                 c2.weight.grad.float(), b2.weight.grad.float()]
        return out.float(), grads, hip.XF_COUNT[0] - n0
    finally:
        hip.FUSE_XF, hip.CONV_FORCE_CFG, hip.WGRAD_STAGES, hip.XF_MAX_REP = keep


@pytest.mark.parametrize("case", [
    # n, cin, hw, cmid, kernel, stride, act, fused expected
    (4, 256, 28, 64, 3, 1, "relu", True),    # bn1 -> conv2 (3x3, padded taps stay zero)
    (4, 128, 28, 128, 3, 2, "relu", True),   # bn1 -> strided conv2 (downsampling block)
    (4, 64, 14, 64, 1, 1, "relu", True),     # bn2 -> conv3 (1x1)
    (2, 256, 7, 512, 3, 1, "relu", True),    # 7x7 map, partial row tiles
    (3, 64, 15, 128, 3, 1, None, True),      # odd pixel count, no activation
    (4, 64, 14, 96, 3, 1, "relu", False),    # 96 channels: no uniform k-steps -> materialised, same result
])
def test_bn_apply_fused_into_consumer_conv(case):
    """Forward / wgrad with the fused BN-apply operand map (XF) against the unfused path (bn_apply writes
    act(bn(y)), plain GEMMs): same outputs and gradients to bf16 accuracy, and the fused path really taken
    (or, for an ineligible consumer, the deferred output materialised)."""
    hip = _hip()
    n, cin, hw, cmid, k, stride, act, fused = case
    o0, g0, k0 = _xf_block(hip, n, cin, hw, cmid, k, stride, act, False)
    o1, g1, k1 = _xf_block(hip, n, cin, hw, cmid, k, stride, act, True)
    assert k0 == 0 and k1 == (1 if fused else 0), (k0, k1)
    assert rel_err(o1, o0) < 2e-2, rel_err(o1, o0)
    for a_, b_ in zip(g1, g0):
        assert rel_err(a_, b_) < 2e-2, rel_err(a_, b_)
        assert mean_err(a_, b_) < 5e-3, mean_err(a_, b_)


def test_bn_apply_fused_every_kernel_variant():
    """Every conv configuration with a fused A-operand variant and every wgrad ring / tile variant with a
    fused X form (256 channels on both convs: the 256 x 256 wgrad tiles qualify), against the unfused path."""
    hip = _hip()
    case = (2, 128, 12, 256, 3, 1, "relu")
    _o, g0, _ = _xf_block(hip, *case, xf_on=False, cout=256)
    ran = 0
    for i in range(len(hip.conv_cfgs())):
        if not hip.C.conv_cfg_has_xa(i):
            continue
        for wst in (1, 2, 3, 4, 7, 8, 9):
            if not hip.C.conv_wgrad_has_xf(wst):
                continue
            o1, g1, k1 = _xf_block(hip, *case, xf_on=True, cout=256, cfg=i, wstages=wst)
            assert k1 == 1
            for a_, b_ in zip(g1, g0):
                assert rel_err(a_, b_) < 2e-2, (i, wst, rel_err(a_, b_))
            ran += 1
    assert ran >= 40


def test_resnet_bottleneck_defers_bn_apply():
    """A ResNet-50 bottleneck in training on the HIP path: bn1 and bn2 outputs are deferred (both consumer
    convs read y through the fused map), and the block's output / gradients match the unfused run."""
    hip = _hip()
    from pytorch_imageclassification_distributed_amd.models.resnet import Bottleneck
    torch.manual_seed(3)
    down = nn.Sequential(nn.Conv2d(256, 512, 1, 2, bias=False), nn.BatchNorm2d(512))
    blk = Bottleneck(256, 128, stride=2, downsample=down).to(DEV).to(memory_format=CL)
    x = torch.randn(4, 256, 28, 28, device=DEV).to(torch.bfloat16).contiguous(memory_format=CL)
    res = []
    for on in (False, True):
        keep = hip.FUSE_XF, hip.XF_MAX_REP, hip.SIBLINGS
        # (the per-branch heads: merged sibling heads (SIBLINGS) write their outputs instead of deferring them)
        hip.FUSE_XF, hip.XF_MAX_REP, hip.SIBLINGS = on, 10 ** 6, False
        try:
            b = copy.deepcopy(blk)
            xb = x.clone().requires_grad_(True)
            n0 = hip.XF_COUNT[0]
            out = b(xb)
            out.float().square().mean().backward()
            torch.cuda.synchronize()
            res.append((out.float(), xb.grad.float(), b.conv2.weight.grad.float(), b.conv3.weight.grad.float(),
                        hip.XF_COUNT[0] - n0))
        finally:
            hip.FUSE_XF, hip.XF_MAX_REP, hip.SIBLINGS = keep
    assert res[0][-1] == 0 and res[1][-1] == 2, (res[0][-1], res[1][-1])
    for a_, b_ in zip(res[1][:-1], res[0][:-1]):
        assert rel_err(a_, b_) < 2e-2, rel_err(a_, b_)


@pytest.mark.parametrize("block,expect", [("A", 1), ("C128", 6), ("C160", 0), ("D", 4), ("E", 1)])
def test_inception_defers_chain_bn_apply(block, expect):
    """Inception blocks: every chain-internal BN output is deferred; consumers with 64-multiple input
    channels read it through the fused map, the others (48 / 96 / 160 channels) materialise it.  Output and
    gradients against the unfused run."""
    hip = _hip()
    from pytorch_imageclassification_distributed_amd.models import inception as inc
    torch.manual_seed(5)
    mk = {"A": (lambda: inc.InceptionA(192, 32), 192, 35), "C128": (lambda: inc.InceptionC(768, 128), 768, 17),
          "C160": (lambda: inc.InceptionC(768, 160), 768, 17), "D": (lambda: inc.InceptionD(768), 768, 17),
          "E": (lambda: inc.InceptionE(1280), 1280, 8)}[block]
    blk = mk[0]().to(DEV).to(memory_format=CL)
    x = torch.randn(4, mk[1], mk[2], mk[2], device=DEV).to(torch.bfloat16).contiguous(memory_format=CL)
    res = []
    for on in (False, True):
        keep = hip.FUSE_XF, hip.XF_MAX_REP, hip.SIBLINGS
        hip.FUSE_XF, hip.XF_MAX_REP, hip.SIBLINGS = on, 10 ** 6, False
        try:
            b = copy.deepcopy(blk)
            xb = x.clone().requires_grad_(True)
            n0 = hip.XF_COUNT[0]
            out = b(xb)
            out.float().square().mean().backward()
            torch.cuda.synchronize()
            wg = [m.weight.grad.float() for m in b.modules() if isinstance(m, nn.Conv2d)]
            res.append((out.float(), xb.grad.float(), wg, hip.XF_COUNT[0] - n0))
        finally:
            hip.FUSE_XF, hip.XF_MAX_REP, hip.SIBLINGS = keep
    assert res[0][3] == 0 and res[1][3] == expect, (res[0][3], res[1][3])
    assert rel_err(res[1][0], res[0][0]) < 2e-2
    assert rel_err(res[1][1], res[0][1]) < 3e-2, rel_err(res[1][1], res[0][1])
    for a_, b_ in zip(res[1][2], res[0][2]):
        assert rel_err(a_, b_) < 3e-2, rel_err(a_, b_)


@pytest.mark.parametrize("path", ["bn_stats", "conv_epilogue"])
def test_bn_statistics_large_mean(path):
    """BN training statistics at |mean| / std ~ 20 (about as large as bf16 activations can carry the
    spread): the partial sums are taken about the running mean (ops/hip.py stat_shift), so the variance
    does not cancel.  The batch mean / variance (read back from the running-statistics update) against
    fp64 statistics of the same bf16 values, for the standalone statistics pass and the conv epilogue."""
    hip = _hip()
    torch.manual_seed(41)
    n, c, hw = 16, 128, 28

    def run(shift_on):
        keep = hip.SHIFT_STATS
        hip.SHIFT_STATS = shift_on
        try:
            bn = nn.BatchNorm2d(c, momentum=1.0).to(DEV)  # running stats = this batch's statistics
            with torch.no_grad():
                bn.running_mean.fill_(60.0)  # steady state: the pivot tracks the batch mean
            if path == "bn_stats":
                y = (60.0 + 3.0 * torch.randn(n, c, hw, hw, device=DEV)).to(torch.bfloat16)
                y = y.contiguous(memory_format=CL)
                hip.BNActFn.apply(y, bn.weight, bn.bias, None, bn, None, False, None, None, None, None,
                                  hip.stat_shift(bn))
                yref = y
            else:
                conv = nn.Conv2d(64, c, 1, bias=False).to(DEV).to(memory_format=CL)
                with torch.no_grad():
                    conv.weight.copy_(bf(1.0 / 64 + 0.05 * torch.randn_like(conv.weight)))
                x = bf(60.0 + 8.0 * torch.randn(n, 64, hw, hw, device=DEV)).to(torch.bfloat16)
                x = x.contiguous(memory_format=CL)
                hip.conv_bn_act(x, conv, bn, None, None)
                yref = conv(x.float()).to(torch.bfloat16)  # the conv output as the HIP path stores it
            torch.cuda.synchronize()
            yd = yref.double()
            mu = yd.mean((0, 2, 3))
            var = yd.var((0, 2, 3), unbiased=True)
            assert (mu.abs() / var.sqrt()).median() > 8, "the case must have a large mean / std"
            e_mu = ((bn.running_mean.double() - mu).abs() / var.sqrt()).max().item()
            e_var = ((bn.running_var.double() - var).abs() / var).max().item()
            return e_mu, e_var
        finally:
            hip.SHIFT_STATS = keep

    (m1, v1), (m0, v0) = run(True), run(False)
    print(f"{path}: mean err/std {m1:.2e} (unshifted {m0:.2e}), var rel err {v1:.2e} (unshifted {v0:.2e})")
    assert m1 < 1e-3 and v1 < 2e-3, (m1, v1)
    if path == "bn_stats":  # same bf16 values on both sides: the shift must not lose accuracy
        assert v1 <= v0 * 1.5 + 1e-6
    # (the conv epilogue sums the fp32 accumulators before their bf16 rounding, the reference the rounded
    # output: ~1e-5 either way, which is that rounding, not the summation)


@pytest.mark.parametrize("shape", [(3, 38, 22), (1, 299, 299), (5, 37, 21)])
@pytest.mark.parametrize("s2d,affine", [(False, None), (False, "inception"), (True, None)])
def test_input_u8_one_pass(s2d, affine, shape):
    """input_from_u8 (one kernel: uint8 NHWC -> bf16 model input) against the reference normalisation
    (data/folder.py normalize = reference dp/loader.py:86-91) in fp32, then the model's affine (Inception
    transform_input) and the layout the old two-pass path produced (prepare_input / prepare_input_s2d)."""
    import numpy as np

    from pytorch_imageclassification_distributed_amd.data.folder import IMAGENET_MEAN, IMAGENET_STD, normalize
    from pytorch_imageclassification_distributed_amd.models.inception import Inception3
    hip = _hip()
    torch.manual_seed(0)
    n, h, w = shape  # odd pixel counts (Inception's 299 x 299, partial batches) and odd sizes for the s2d stem
    u8 = torch.randint(0, 256, (n, h, w, 3), dtype=torch.uint8)
    ref = torch.from_numpy(np.stack([normalize(u8[i].numpy().astype(np.float32)) for i in range(n)]))  # NHWC fp32
    ref = ref.permute(0, 3, 1, 2).contiguous()  # NCHW
    sc = sh = None
    if affine == "inception":
        sc, sh = Inception3.TRANSFORM_SCALE, Inception3.TRANSFORM_SHIFT
        ref = ref * torch.tensor(sc).view(1, 3, 1, 1) + torch.tensor(sh).view(1, 3, 1, 1)
    y = hip.input_from_u8(u8.to(DEV), (s2d, sc, sh), IMAGENET_MEAN, IMAGENET_STD)
    if s2d and h % 2 == 0 and w % 2 == 0:
        assert y._imgcls_s2d == (h, w) and tuple(y.shape) == (n, 16, h // 2, w // 2)
        want = torch.empty_like(y)
        hip.C.prepare_input_s2d(ref.to(DEV), want, n, h, w)
    else:
        assert y._imgcls_prepared and tuple(y.shape) == (n, 8, h, w) and y.is_contiguous(memory_format=CL)
        want = torch.zeros(n, 8, h, w, device=DEV)
        want[:, :3] = ref.to(DEV)
    # one bf16 rounding of the same fp32 value (the affine's operation order differs): <= 1 ulp apart
    d = (y.float() - want.float()).abs()
    assert (d <= want.float().abs() * 2 ** -7 + 1e-6).all(), d.max()


def test_input_u8_resnet_forward_matches_fp32_input():
    """A ResNet fed the loader-converted (space-to-depth) batch computes what it computes from the fp32 NCHW
    batch of the same images (eval mode, same weights): the s2d marker routes around prepare_input_s2d."""
    from pytorch_imageclassification_distributed_amd.data.folder import IMAGENET_MEAN, IMAGENET_STD
    from pytorch_imageclassification_distributed_amd.models import Classifier
    hip = _hip()
    torch.manual_seed(0)
    m = Classifier("resnet18", 7).to(DEV).eval()
    u8 = torch.randint(0, 256, (4, 64, 64, 3), dtype=torch.uint8, device=DEV)
    x32 = torch.empty(4, 3, 64, 64, device=DEV)
    hip.C.normalize_u8(u8, x32, list(IMAGENET_MEAN), list(IMAGENET_STD))
    spec = m.encoder.input_spec()
    assert spec[0] is True
    with torch.no_grad():
        a = m(hip.input_from_u8(u8, spec, IMAGENET_MEAN, IMAGENET_STD)).float()
        b = m(x32).float()
    assert rel_err(a, b) < 2e-2


@pytest.mark.parametrize("rows,c", [(4099, 256), (1000, 2048), (777, 64), (301, 1152), (20000, 128)])
def test_bn_backward_reduce_walks(rows, c):
    """bn_bwd_reduce (plain, ReLU, residual + ReLU with dz written) and bn_stats under the grid-stride walk
    (default) and the block-contiguous walk, with and without non-temporal loads: partial sums against fp64
    torch, dz bitwise."""
    hip = _hip()
    torch.manual_seed(6)
    y = (torch.randn(rows, c, device=DEV) * 2).to(torch.bfloat16)
    res = torch.randn(rows, c, device=DEV).to(torch.bfloat16)
    g = torch.randn(rows, c, device=DEV).to(torch.bfloat16)
    coef = torch.cat([torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV),
                      torch.randn(c, device=DEV) * 0.1, torch.rand(c, device=DEV) + 0.5])
    sc, sh, mu, iv = coef.view(4, c).double()
    yd, rd, gd = y.double(), res.double(), g.double()
    grp = 16
    dz_ref = None
    try:
        for red_walk, nt in ((1, -1), (0, -1), (1, 0), (0, 0)):
            hip.C.bn_set_stream(1024, nt, -1, -1, 0, 0, red_walk)
            for act, use_res in ((0, False), (1, False), (1, True)):
                part = torch.zeros(grp * 2 * c, dtype=torch.float32, device=DEV)
                dz = torch.empty_like(y) if use_res else None
                hip.C.bn_bwd_reduce(g, y, coef, res if use_res else None, dz, rows, c, act, part, grp)
                torch.cuda.synchronize()
                z = yd * sc + sh + (rd if use_res else 0)
                dzw = gd * (z > 0) if act else gd
                want = torch.stack([dzw.sum(0), (dzw * (yd - mu) * iv).sum(0)])
                got = part.view(grp, 2, c).double().sum(0)
                assert rel_err(got.float(), want.float()) < 1e-3, (red_walk, nt, act, use_res)
                if use_res:
                    if dz_ref is None:
                        dz_ref = dz
                    assert torch.equal(dz, dz_ref)
            # forward statistics pass (sums of y - shift and their squares) under the same walk
            part = torch.zeros(grp * 2 * c, dtype=torch.float32, device=DEV)
            shift = torch.randn(c, device=DEV) * 0.1
            hip.C.bn_stats(y, rows, c, part, grp, shift)
            torch.cuda.synchronize()
            d = yd - shift.double()
            want = torch.stack([d.sum(0), (d * d).sum(0)])
            assert rel_err(part.view(grp, 2, c).double().sum(0).float(), want.float()) < 1e-3, (red_walk, nt)
    finally:
        hip.C.bn_set_stream(1024, -1, 2, 2, 1, 4, 1)  # the defaults


@pytest.mark.parametrize("rows,c", [(4099, 256), (1000, 2048), (777, 64), (301, 1152)])
def test_bn_streaming_passes_every_grid_and_nt(rows, c):
    """bn_apply (+residual +ReLU mask, and plain) and bn_bwd_elemt (all four modes) under every streaming setting
    (flat one-vector-per-thread form; U-row kernels with the block-contiguous or grid-stride walk, grid capped at
    64 / 1024 / grid_chan's; non-temporal never / always) against fp32 torch: the walk, grid and cache hint change
    the access pattern, never a value - all settings are bitwise identical."""
    hip = _hip()
    torch.manual_seed(5)
    y = bf(torch.randn(rows, c, device=DEV) * 2).to(torch.bfloat16)
    res = bf(torch.randn(rows, c, device=DEV)).to(torch.bfloat16)
    g = bf(torch.randn(rows, c, device=DEV)).to(torch.bfloat16)
    coef = torch.cat([torch.rand(c, device=DEV) + 0.5, torch.randn(c, device=DEV),
                      torch.randn(c, device=DEV) * 0.1, torch.rand(c, device=DEV) + 0.5])
    kk = torch.randn(2 * c, device=DEV) * 0.1
    sc, sh, mu, iv = coef.view(4, c)
    yf, rf, gf = y.float(), res.float(), g.float()
    z_res = yf * sc + sh + rf
    want_apply_res = torch.relu(z_res)
    want_apply = torch.relu(yf * sc + sh)
    xhat = (yf - mu) * iv
    k1, k2 = kk.view(2, c)

    def elemt(gz):
        return sc * (gz - k1 - xhat * k2)
    want_bwd = {0: elemt(gf), 1: elemt(gf * (yf * sc + sh > 0)), 2: elemt(gf * (z_res > 0)), 3: elemt(gf)}
    outs = []
    try:
        for grid, nt, walk, wb, fu in ((1024, -1, 2, 1, 1), (1024, -1, 2, 1, 2), (1024, 0, 2, 1, 4),
                                       (1024, 256, 2, 2, 1), (1024, -1, 2, 2, 2), (1024, -1, 2, 2, 4),
                                       (1024, -1, 2, 3, 1), (1024, -1, 2, 3, 4), (1024, 256, 1, 1, 1),
                                       (0, 0, 1, 1, 1), (1024, -1, 1, 1, 1), (64, -1, 1, 1, 1), (64, 0, 0, 0, 1)):
            hip.C.bn_set_stream(grid, nt, walk, wb, fu, fu)
            o1 = torch.empty_like(y)
            mask = torch.zeros(rows * c // 8, dtype=torch.uint8, device=DEV)
            hip.C.bn_apply(y, coef, res, o1, rows, c, c, 0, 1, None, None, mask=mask)
            o2 = torch.empty_like(y)
            hip.C.bn_apply(y, coef, None, o2, rows, c, c, 0, 1, None, None)
            bw = {}
            for mode in range(4):
                d = torch.empty_like(y)
                hip.C.bn_bwd_elemt(None if mode == 0 else g, y, coef, kk, res if mode == 2 else None,
                                   g if mode == 0 else None, d, rows, c, 0 if mode == 3 else 1, 0)
                bw[mode] = d
            torch.cuda.synchronize()
            assert rel_err(o1.float(), want_apply_res) < 1e-2 and rel_err(o2.float(), want_apply) < 1e-2
            bits = torch.stack([(mask >> k) & 1 for k in range(8)], 1).view(rows, c).bool()
            assert torch.equal(bits, z_res.view(rows, c) > 0) or (bits != (z_res > 0)).float().mean() < 1e-4
            for mode in range(4):
                assert rel_err(bw[mode].float(), want_bwd[mode]) < 1e-2, (grid, nt, walk, wb, fu, mode)
            outs.append([o1, o2, mask] + [bw[m] for m in range(4)])
    finally:
        hip.C.bn_set_stream(1024, -1, 2, 2, 1, 4, 1)  # the defaults
    for o in outs[1:]:
        for a_, b_ in zip(o, outs[0]):
            assert torch.equal(a_, b_)
