"""GPU distributed path, 2 ranks sharing one GPU (gloo transport), HIP kernels.

W=2 ranks with half batches, SyncBN on and the bucketed GradReducer must give the
same gradients as one process on the full batch (bf16 tolerance).  On an 8-GPU
node the identical code runs over RCCL; this test exercises it on a 1-GPU box.
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


def _worker(rank, world, port, out_dir, name="resnet18", damp=True, det=False, direct=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    # Fixed kernel choices (shape heuristic, one weight-gradient plan) in every process: ResNet-50 train-mode
    # gradients at random init are chaotic - 0.1 % fp32 weight noise alone drops some BN-bias gradient
    # cosines to 0.14-0.28 on the CPU fp32 path (scripts/cpu_weight_noise.py,
    # profiles/history/r2_cpu_weight_noise_resnet50.txt) - so per-process timed tuner picks (two ranks contending
    # for one GPU time the candidates differently) made the comparison flaky (scripts/tune_random_choices.py).
    os.environ.update(IMGCLS_CONV_STAGES="0", IMGCLS_WGRAD_BLOCKS="512", IMGCLS_WGRAD_STAGES="2",
                      IMGCLS_DIRECT_CONV="1" if direct else "0")
    import torch.nn.functional as F
    from pytorch_imageclassification_distributed_amd.models import Classifier
    from pytorch_imageclassification_distributed_amd.ops import functional as Fx
    from pytorch_imageclassification_distributed_amd.parallel import (GradReducer, convert_sync_batchnorm, destroy,
                                                                      init_distributed)
    ctx = init_distributed(device="cuda", backend="gloo")
    dev = ctx.device
    from pytorch_imageclassification_distributed_amd.ops import hip
    if det:
        hip.set_deterministic(True)
    if direct:  # every eligible 3x3 conv (fwd and fused dgrad) on the 64 x 64 direct variant
        hip.DIRECT_FORCE = 3
    torch.manual_seed(0)
    x = torch.randn(16, 3, 64, 64, device=dev).to(torch.bfloat16).float()
    y = torch.randint(0, 7, (16,), device=dev)

    def model():
        torch.manual_seed(1)
        m = Classifier(name, 7)
        if damp:
            with torch.no_grad():  # damp the Bottleneck residual branches (the chaos above); grads stay non-zero
                for n, p in m.named_parameters():
                    if n.endswith("bn3.weight"):
                        p.mul_(0.1)
        return m.to(dev).to(memory_format=torch.channels_last)

    m = model()
    convert_sync_batchnorm(m)
    red = GradReducer(m, bucket_cap_mb=4, first_bucket_mb=1)
    xs, ys = x[rank * 8:(rank + 1) * 8], y[rank * 8:(rank + 1) * 8]
    early0 = hip.SYNCBN_EARLY_COUNT[0]
    Fx.cross_entropy(m(xs), ys).backward()
    scale = red.finish()
    assert hip.SYNCBN_EARLY_COUNT[0] > early0  # fused links started their SyncBN all-reduce early
    grads = {n: (p.grad * scale).float().cpu() for n, p in m.named_parameters()}
    rm = m.encoder.bn1.running_mean.cpu()
    if rank == 0:
        ref = model()
        Fx.cross_entropy(ref(x), y).backward()
        for n, p in ref.named_parameters():
            cos = F.cosine_similarity(p.grad.float().cpu().flatten(), grads[n].flatten(), dim=0).item()
            assert cos > 0.97, (n, cos)
        assert torch.allclose(ref.encoder.bn1.running_mean.cpu(), rm, rtol=2e-2, atol=2e-3)
    destroy()


@pytest.mark.parametrize("name,damp,det,direct", [
    ("resnet18", False, False, False),
    ("resnet50", True, False, False),
    ("resnet50", True, False, True),   # direct (halo-tile) 3x3 convs and their fused dgrad on the SyncBN path
    ("resnet50", False, True, False),  # undamped, deterministic mode in both runs (no atomics-order noise)
])
def test_two_ranks_one_gpu_matches_full_batch(tmp_path, name, damp, det, direct):
    """ResNet-18 (BasicBlock) and ResNet-50 (Bottleneck: fused BN-backward links whose SyncBN
    all-reduce is launched early by the consuming conv, residual gradient slots)."""
    mp.spawn(_worker, args=(2, _port(), str(tmp_path), name, damp, det, direct), nprocs=2, join=True)
