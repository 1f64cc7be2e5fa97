"""Conditioning of random-init ResNet-50 train-mode gradients, on the CPU fp32 path (no HIP kernels).

Computes every parameter gradient of the reference model (Classifier + MLP head, 7 classes, weighted CE,
train-mode BN) for one batch, then again after multiplying every weight by (1 + eps * N(0, 1)), and prints
the per-parameter gradient cosine between the two runs (worst first).  A well-conditioned network keeps
every cosine near 1 for eps = 1e-3; this one does not - the justification for damping the Bottleneck
branches in tests/test_gpu_multirank.py (docs/DESIGN.md, "Random-init gradients are chaotic").

    python scripts/cpu_weight_noise.py [eps=1e-3] [trials=3] [model=resnet50]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from pytorch_imageclassification_distributed_amd.models import Classifier
from pytorch_imageclassification_distributed_amd.ops import functional as Fx

eps = float(sys.argv[1]) if len(sys.argv) > 1 else 1e-3
trials = int(sys.argv[2]) if len(sys.argv) > 2 else 3
name = sys.argv[3] if len(sys.argv) > 3 else "resnet50"
torch.set_num_threads(min(8, os.cpu_count() or 1))
torch.manual_seed(0)
x = torch.randn(8, 3, 64, 64)
y = torch.randint(0, 7, (8,))
w = torch.tensor([3, 3, 10, 1, 4, 4, 5], dtype=torch.float32)


def grads(noise_seed=None):
    torch.manual_seed(1)
    m = Classifier(name, 7)
    if noise_seed is not None:
        g = torch.Generator().manual_seed(noise_seed)
        with torch.no_grad():
            for p in m.parameters():
                p.mul_(1 + eps * torch.randn(p.shape, generator=g))
    loss = Fx.cross_entropy(m(x), y, w)
    loss.backward()
    return loss.item(), {n: p.grad.flatten().clone() for n, p in m.named_parameters()}


l0, g0 = grads()
print(f"model {name}, batch 8 @ 64x64, fp32 CPU, weight noise eps={eps}; base loss {l0:.6f}")
for t in range(trials):
    lt, gt = grads(100 + t)
    cos = {n: F.cosine_similarity(gt[n], g0[n], dim=0).item() for n in g0}
    worst = sorted(cos.items(), key=lambda kv: kv[1])
    below = sum(1 for v in cos.values() if v < 0.97)
    print(f"trial {t}: loss {lt:.6f}; {below}/{len(cos)} parameters below cosine 0.97; worst:")
    for n, v in worst[:8]:
        print(f"    {v:8.4f}  {n}")
    head = [v for n, v in cos.items() if ".fc." in n or n.startswith("encoder.fc")]
    print(f"    head (fc.*) min cosine {min(head):.5f}")
