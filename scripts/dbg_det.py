import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pytorch_imageclassification_distributed_amd.models import Classifier
dev = "cuda"
torch.manual_seed(0)
m = Classifier(os.environ.get("M", "efficientnet-b0"), 5).to(dev).to(memory_format=torch.channels_last).train()
x = torch.randn(4, 3, 64, 64, device=dev)
params = [p for p in m.parameters()]
names = [n for n, _ in m.named_parameters()]
def run():
    for p in params: p.grad = None
    torch.manual_seed(1)
    out = m(x).float()
    loss = out.square().mean()
    loss.backward()
    return out.detach().clone(), [p.grad.clone() for p in params]
o1, g1 = run()
for it in range(6):
    o, g = run()
    worst = max(((a - b).abs().max().item() / (a.abs().max().item() + 1e-12), n) for n, a, b in zip(names, g1, g))
    print(f"run {it+2}: out diff {(o - o1).abs().max().item():.3g}  worst grad {worst[0]:.3g} {worst[1]}", flush=True)
