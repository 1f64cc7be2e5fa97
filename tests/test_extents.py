"""Host-side launch-extent checks (csrc/extents.h) on the CPU.

Every conv launch passes ``conv_gemm_extent_error`` / ``conv_wgrad_extent_error`` in the bindings before it is
enqueued (tuner candidates included: they go through the same bindings).  Here the same functions are swept with
integers only, no GPU:

* every GEMM convolution of five models (ResNet-18 @32 / @224, ResNet-50 @224, Inception-v3 @299,
  EfficientNet-B0 @224, EfficientNet-B3 @300) at per-GPU batches 1, 4, 128 and 1024: the forward launch, every
  sub-pixel data-gradient phase, and the weight gradient under every split plan the tuner can pick (each
  variant's output tile -> split count), with the tensor sizes the launchers allocate;
* the test shapes of tests/test_hip_ops.py, including the pointwise 144 -> 24 conv at 1,200 pixels whose
  backward preceded the round-5 transient fault (profiles/r13o_gpu_suite_transient_fault.txt);
* negative cases: each bound, violated on purpose, is reported.

Reference workload: /root/reference/nn/classifier.py:14-23 (the model zoo), train.py:110 (image sizes).
"""
import pytest
import torch

from pytorch_imageclassification_distributed_amd import _ext
from pytorch_imageclassification_distributed_amd.ops import functional as Fx

C = _ext.load()

CONV_FIELDS = ("M Ncols K CA GH GW IH IW sA ldb OH OW so oh0 ow0 ldc c_off ntaps a_numel b_numel c_numel max_tb "
               "stats_numel stats_groups part_numel part_groups coef_numel mask_numel bias_numel").split()
WGRAD_FIELDS = ("M Cout Cin Ntot OH OW IH IW KW k_per_split splits dy_numel x_numel dw_numel ws_numel tile_rows "
                "tile_cols").split()
G_STATS = 64


def conv_check(**kw):
    d = dict(stats_numel=-1, stats_groups=1, part_numel=-1, part_groups=1, coef_numel=-1, mask_numel=-1,
             bias_numel=-1)
    d.update(kw)
    return C.conv_extent_check([int(d[f]) for f in CONV_FIELDS])


def wgrad_check(**kw):
    return C.wgrad_extent_check([int(kw[f]) for f in WGRAD_FIELDS])


class _Geom:
    """ops/_hip/gemm.py ConvGeom of a recorded (conv, input shape), without touching a device."""

    def __init__(self, conv, shape):
        from pytorch_imageclassification_distributed_amd.ops._hip.gemm import ConvGeom
        self.g = ConvGeom(torch.empty(shape, device="meta"), conv)


def _record(model_name, size, num_classes=7):
    """(conv module, input shape) of every GEMM convolution one forward runs (CPU path, batch 1)."""
    from pytorch_imageclassification_distributed_amd.models import Classifier
    torch.manual_seed(0)
    net = Classifier(model_name, num_classes).eval()
    seen, orig = [], Fx._torch_conv

    def spy(x, conv):
        if conv.groups == 1:  # depthwise convs run the dwconv kernels, not the GEMM
            seen.append((conv, tuple(x.shape)))
        return orig(x, conv)

    Fx._torch_conv = spy
    try:
        with torch.no_grad():
            net(torch.zeros(1, 3, size, size))
    finally:
        Fx._torch_conv = orig
    assert seen, model_name
    return seen


def _launches(conv, shape, batch):
    """Every conv_gemm / conv_wgrad argument set the HIP launchers derive for this conv at ``batch``."""
    from pytorch_imageclassification_distributed_amd.ops._hip import gemm as G
    c = -(-shape[1] // 8) * 8  # the 3-channel image is padded to 8 channels on the device (prepare_input)
    shape = (batch, c) + shape[2:]
    g = _Geom(conv, shape).g
    dh, dw, tb = G._fwd_taps(g)
    x_n, y_n = g.N * g.H * g.W * g.Cx, g.N * g.OH * g.OW * g.Co
    M = g.N * g.OH * g.OW
    rows = [("fwd", dict(M=M, Ncols=g.Co, K=g.T * g.Cx, CA=g.Cx, GH=g.OH, GW=g.OW, IH=g.H, IW=g.W, sA=g.sh,
                         ldb=g.T * g.Cx, OH=g.OH, OW=g.OW, so=1, oh0=0, ow0=0, ldc=g.Co, c_off=0, ntaps=len(dh),
                         a_numel=x_n, b_numel=g.Co * g.T * g.Cx, c_numel=y_n, max_tb=max(tb),
                         stats_numel=2 * G_STATS * g.Co, stats_groups=G_STATS))]
    dx_n = g.N * g.H * g.W * g.Ci
    for ph, pw, gh, gw, pdh, pdw, ptb in G._dgrad_phases(g):
        if g.Ci % 8:  # the image-input conv: no data gradient is ever computed for the input
            break
        if gh <= 0 or gw <= 0 or not ptb:
            continue
        rows.append((f"dgrad{ph}{pw}", dict(
            M=g.N * gh * gw, Ncols=g.Ci, K=len(ptb) * g.Co, CA=g.Co, GH=gh, GW=gw, IH=g.OH, IW=g.OW, sA=1,
            ldb=g.T * g.Co, OH=g.H, OW=g.W, so=g.sh, oh0=ph, ow0=pw, ldc=g.Ci, c_off=0, ntaps=len(ptb),
            a_numel=y_n, b_numel=g.Ci * g.T * g.Co, c_numel=dx_n, max_tb=max(ptb),
            part_numel=2 * G_STATS * g.Ci, part_groups=G_STATS, coef_numel=4 * g.Ci, mask_numel=dx_n // 8)))
    wg = []
    ntot = g.T * g.Cx
    for stages in range(1, 17):
        if stages == 16 and g.Co > 64:
            continue
        tiles = G._wgrad_tiles(g.Co, ntot, stages)
        for target in G.WGRAD_CANDIDATES:
            kps, splits = G._wgrad_split(M, tiles, target)
            tr = 256 if stages in (4, 7, 9, 12, 13, 15) else 32 if stages in (5, 6) else 64 if g.Co <= 64 else 128
            tc = 256 if stages in (4, 7, 9, 13, 14, 16) else 64 if stages in (10, 11, 12) else 128
            wg.append((f"wgrad st{stages} t{target}", dict(
                M=M, Cout=g.Co, Cin=g.Cx, Ntot=ntot, OH=g.OH, OW=g.OW, IH=g.H, IW=g.W, KW=g.kw, k_per_split=kps,
                splits=splits, dy_numel=y_n, x_numel=x_n, dw_numel=g.Co * ntot,
                ws_numel=splits * g.Co * ntot if splits > 1 else -1, tile_rows=tr, tile_cols=tc)))
    return rows, wg


MODELS = [("resnet18", 32), ("resnet18", 224), ("resnet50", 224), ("inceptionv3", 299), ("efficientnet-b0", 224),
          ("efficientnet-b3", 300)]


@pytest.mark.parametrize("model,size", MODELS)
def test_every_model_conv_launch_is_in_bounds(model, size):
    n = 0
    for conv, shape in _record(model, size):
        for batch in (1, 4, 128, 1024):
            rows, wg = _launches(conv, shape, batch)
            for kind, kw in rows:
                err = conv_check(**kw)
                assert err == "", (model, kind, shape, batch, err)
                n += 1
            for kind, kw in wg:
                err = wgrad_check(**kw)
                assert err == "", (model, kind, shape, batch, err)
                n += 1
    assert n > 100


@pytest.mark.parametrize("case", [(2, 16, 40, 40, 96), (2, 24, 28, 28, 144), (3, 144, 20, 20, 24),
                                  (2, 32, 33, 31, 16), (2, 40, 14, 14, 240), (2, 96, 15, 15, 24), (1, 80, 9, 7, 48)])
def test_pointwise_test_shapes_in_bounds(case):
    """tests/test_hip_ops.py PW_CASES: forward, data gradient and every weight-gradient plan of each 1x1 conv
    (case (3, 144, 20, 20, 24) is the one whose backward preceded the round-5 transient fault)."""
    import torch.nn as nn
    n, c, h, w, co = case
    conv = nn.Conv2d(c, co, 1, bias=False)
    rows, wg = _launches(conv, (n, c, h, w), n)
    for kind, kw in rows:
        assert conv_check(**kw) == "", (kind, case)
    for kind, kw in wg:
        assert wgrad_check(**kw) == "", (kind, case)


def _base():
    # a 3x3 stride-1 forward, 2 images of 8x8, 16 -> 32 channels
    return dict(M=128, Ncols=32, K=144, CA=16, GH=8, GW=8, IH=8, IW=8, sA=1, ldb=144, OH=8, OW=8, so=1, oh0=0,
                ow0=0, ldc=32, c_off=0, ntaps=9, a_numel=2 * 64 * 16, b_numel=32 * 144, c_numel=2 * 64 * 32, max_tb=8)


@pytest.mark.parametrize("change,needle", [
    (dict(c_numel=2 * 64 * 32 - 8), "output"),
    (dict(a_numel=64 * 16), "images"),
    (dict(b_numel=32 * 144 - 16), "B is shorter"),
    (dict(OH=7), "height"),
    (dict(ow0=1), "width"),
    (dict(c_off=8), "channel slice"),
    (dict(K=128), "K != taps"),
    (dict(stats_numel=2 * 64 * 32 - 1, stats_groups=64), "statistics"),
    (dict(part_numel=10, part_groups=64), "partials"),
    (dict(coef_numel=3 * 32), "coefficients"),
    (dict(mask_numel=2 * 64 * 32 // 8 - 1), "mask"),
    (dict(bias_numel=31), "bias"),
])
def test_conv_extent_violations_are_reported(change, needle):
    assert conv_check(**_base()) == ""
    kw = _base()
    kw.update(change)
    assert needle in conv_check(**kw)


def test_conv_extent_concat_slice_and_partial_grid():
    # an Inception concat slice: ldc = the block's total channels, c_off = the branch's offset
    kw = _base()
    kw.update(ldc=96, c_off=64, c_numel=2 * 64 * 96)
    assert conv_check(**kw) == ""
    kw.update(c_off=72)
    assert "channel slice" in conv_check(**kw)
    # a GEMM view with fewer rows than one image (benchmarks/gemm_ref.py style M x 1 grid)
    kw = dict(M=100, Ncols=64, K=64, CA=64, GH=100, GW=1, IH=100, IW=1, sA=1, ldb=64, OH=100, OW=1, so=1, oh0=0,
              ow0=0, ldc=64, c_off=0, ntaps=1, a_numel=100 * 64, b_numel=64 * 64, c_numel=100 * 64, max_tb=0)
    assert conv_check(**kw) == ""
    # a stride-2 data-gradient phase (1, 1) of an 8x8 input: a 4x4 grid at rows / columns 1, 3, 5, 7
    kw = dict(M=2 * 16, Ncols=16, K=32, CA=32, GH=4, GW=4, IH=4, IW=4, sA=1, ldb=32, OH=8, OW=8, so=2, oh0=1,
              ow0=1, ldc=16, c_off=0, ntaps=1, a_numel=2 * 16 * 32, b_numel=16 * 32, c_numel=2 * 64 * 16, max_tb=0)
    assert conv_check(**kw) == ""
    kw.update(GH=5, M=2 * 20, IH=5, a_numel=2 * 20 * 32)  # one grid row too many: 4 * 2 + 1 = 9 >= 8
    assert "height" in conv_check(**kw)


def _wbase():
    return dict(M=2 * 64, Cout=32, Cin=16, Ntot=144, OH=8, OW=8, IH=8, IW=8, KW=3, k_per_split=64, splits=2,
                dy_numel=128 * 32, x_numel=2 * 64 * 16, dw_numel=32 * 144, ws_numel=2 * 32 * 144, tile_rows=32,
                tile_cols=128)


@pytest.mark.parametrize("change,needle", [
    (dict(splits=1, ws_numel=-1), "cover"),
    (dict(splits=3, ws_numel=3 * 32 * 144), "empty split"),
    (dict(dy_numel=128 * 32 - 8), "dY"),
    (dict(x_numel=64 * 16), "X holds"),
    (dict(dw_numel=32 * 144 - 4), "dW"),
    (dict(ws_numel=32 * 144), "workspace"),
    (dict(Ntot=140), "Ntot"),
    (dict(M=100), "whole number"),
])
def test_wgrad_extent_violations_are_reported(change, needle):
    assert wgrad_check(**_wbase()) == ""
    kw = _wbase()
    kw.update(change)
    assert needle in wgrad_check(**kw)
