import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pytorch_imageclassification_distributed_amd.ops import hip
C = hip.C
torch.manual_seed(0)
dev = "cuda"
for (M, N, K, bias, relu) in [(4, 5, 1280, True, False), (256, 128, 2048, True, True), (4, 48, 1152, True, False),
                              (256, 7, 32, True, False), (128, 2048, 256, False, False)]:
    a = torch.randn(M, K, device=dev); w = torch.randn(N, K, device=dev); b = torch.randn(N, device=dev) if bias else None
    out = torch.empty(M, N, device=dev)
    hip._mm(a, w, out, M, N, K, K, 1, 1, K, bias=b, relu=relu)
    ref = a @ w.t() + (b if bias else 0)
    ref = ref.relu() if relu else ref
    torch.cuda.synchronize()
    print("sgemm", M, N, K, (out - ref).abs().max().item() / ref.abs().max().item())
for (M, N) in [(4, 1152), (256, 128), (256, 7), (4, 48)]:
    x = torch.randn(M, N, device=dev); o = torch.empty(N, device=dev)
    C.colsum(x, None, o, M, N, N, False)
    torch.cuda.synchronize()
    print("colsum", M, N, (o - x.sum(0)).abs().max().item())
from pytorch_imageclassification_distributed_amd.models import Classifier
m = Classifier("efficientnet-b0", 5).to(dev).to(memory_format=torch.channels_last).train()
x = torch.randn(4, 3, 64, 64, device=dev)
params = [p for p in m.parameters()]
names = [n for n, _ in m.named_parameters()]
def run():
    for p in params: p.grad = None
    torch.manual_seed(1)
    m(x).float().square().mean().backward()
    return [p.grad.clone() for p in params]
g1 = run(); g2 = run(); g3 = run()
for n, a, b, c in zip(names, g1, g2, g3):
    d12 = (a - b).abs().max().item() / (a.abs().max().item() + 1e-12)
    d23 = (b - c).abs().max().item() / (b.abs().max().item() + 1e-12)
    if d12 > 1e-2 or d23 > 1e-2:
        print("MISMATCH", n, tuple(a.shape), f"{d12:.3g} {d23:.3g}")
print("done")
