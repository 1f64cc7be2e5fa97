"""Poison the caching allocator with NaN, then find the first module whose output is non-finite
(an uninitialised read in some kernel)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pytorch_imageclassification_distributed_amd.models import Classifier
dev = "cuda"
torch.manual_seed(0)
name = os.environ.get("M", "efficientnet-b0")
m = Classifier(name, 5).to(dev).to(memory_format=torch.channels_last).train()
x = torch.randn(4, 3, 64, 64, device=dev)

def poison():
    small = [torch.full((s,), float("nan"), device=dev) for s in (1024, 4096, 16384, 65536, 131072) for _ in range(64)]
    big = [torch.full((n,), float("nan"), device=dev) for n in (2**22, 2**24, 2**26)]
    del small, big
    torch.cuda.synchronize()

bad = []
def hook(mod, inp, out):
    outs = out if isinstance(out, (tuple, list)) else (out,)
    for o in outs:
        if torch.is_tensor(o) and o.is_floating_point() and not torch.isfinite(o).all().item():
            bad.append(mod._dbg_name)
for n, mod in m.named_modules():
    mod._dbg_name = n
    mod.register_forward_hook(hook)

for it in range(3):
    for p in m.parameters(): p.grad = None
    poison()
    torch.manual_seed(1)
    out = m(x).float()
    print(f"iter {it}: first non-finite module outputs: {bad[:5]}", flush=True)
    bad.clear()
    out.square().mean().backward()
    nf = [n for n, p in m.named_parameters() if p.grad is None or not torch.isfinite(p.grad).all().item()]
    print(f"iter {it}: params with non-finite/missing grads: {len(nf)} first {nf[-5:]}", flush=True)
