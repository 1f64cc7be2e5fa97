"""Run the same fwd+bwd twice; report per-module forward-output and grad-input divergence
(first modules in execution order whose results differ beyond 1e-3 relative)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pytorch_imageclassification_distributed_amd.models import Classifier
dev = "cuda"
torch.manual_seed(0)
name = os.environ.get("M", "efficientnet-b0")
B, R = int(os.environ.get("B", "8")), int(os.environ.get("R", "128"))
m = Classifier(name, 5).to(dev).to(memory_format=torch.channels_last).train()
x = torch.randn(B, 3, R, R, device=dev)
rec = {}
def fh(mod, inp, out):
    if torch.is_tensor(out):
        rec.setdefault("f", []).append((mod._n, out.detach().float().clone()))
def bh(mod, gin, gout):
    g = gout[0]
    if torch.is_tensor(g):
        rec.setdefault("b", []).append((mod._n, g.detach().float().clone()))
for n, mod in m.named_modules():
    mod._n = n
    if len(list(mod.children())) == 0 or n.endswith("]") or "blocks." in n and n.count(".") == 2:
        mod.register_forward_hook(fh)
        mod.register_full_backward_hook(bh)
def run():
    rec.clear()
    for p in m.parameters(): p.grad = None
    torch.manual_seed(1)
    m(x).float().square().mean().backward()
    return dict(f=list(rec.get("f", [])), b=list(rec.get("b", []))), [p.grad.clone() for p in m.parameters()]
runs = [run() for _ in range(4)]
names = [n for n, _ in m.named_parameters()]
for i in range(1, 4):
    (r0, g0), (ri, gi) = runs[0], runs[i]
    print(f"--- run 0 vs run {i}")
    for kind in ("f", "b"):
        shown = 0
        for (n, a), (_, b) in zip(r0[kind], ri[kind]):
            d = (a - b).abs().max().item() / (a.abs().max().item() + 1e-20)
            if d > 1e-3 and shown < 4:
                print(f"  {kind} {n}: rel {d:.3g} shape {tuple(a.shape)}")
                shown += 1
    cs = []
    for n, a, b in zip(names, g0, gi):
        a64, b64 = a.double().flatten(), b.double().flatten()
        cs.append(((a64 @ b64) / (a64.norm() * b64.norm() + 1e-30)).item())
    worst = sorted(zip(cs, names))[:3]
    print("  worst param cos:", [(round(c, 4), n) for c, n in worst])
