"""Stream-race check: a few deterministic-mode training steps, then one SHA-256 over every
parameter, BN buffer and gradient.

The HIP path runs weight gradients on a side stream, gradient collectives on a comm stream and the input
copies on a copy stream.  A missing stream wait shows up as a result that depends on timing.  Run this
twice, once normally and once with every kernel serialised (``AMD_SERIALIZE_KERNEL=3``, set before the
process touches the GPU): in deterministic mode the digests must be equal
(tests/test_gpu_race.py does exactly that).

    python scripts/race_check.py --model resnet18 --steps 3
    AMD_SERIALIZE_KERNEL=3 python scripts/race_check.py --model resnet18 --steps 3
"""
from __future__ import annotations

import argparse
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet18")
    ap.add_argument("--image-size", type=int, default=64)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    import torch
    from pytorch_imageclassification_distributed_amd.engine import Trainer, build_parser
    from pytorch_imageclassification_distributed_amd.ops import hip
    from pytorch_imageclassification_distributed_amd.parallel import init_distributed
    ctx = init_distributed(device="cuda")
    args = build_parser().parse_args([
        "--synthetic", "--model", a.model, "--image-size", str(a.image_size), "--batchsize", str(a.batch),
        "--num-classes", "7", "--num-workers", "0", "--synthetic-train-size", "8", "--synthetic-val-size", "8",
        "--no-sync-bn", "--lr", "1e-3", "--seed", "3", "--deterministic", "--hip-graph", "off"])
    tr = Trainer(args, ctx)
    hip.set_deterministic(True)
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(a.batch, 3, a.image_size, a.image_size, device="cuda", generator=g)
    y = torch.randint(0, 7, (a.batch,), device="cuda", generator=g)
    tr.net.train()
    for _ in range(a.steps):
        torch.manual_seed(11)
        tr.train_step(x, y)
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for name, t in list(tr.model.state_dict().items()):
        h.update(name.encode())
        h.update(t.detach().float().cpu().numpy().tobytes())
    for p in tr.model.parameters():
        if p.grad is not None:
            h.update(p.grad.detach().float().cpu().numpy().tobytes())
    print(f"race_check {a.model} steps {a.steps} serialize={os.environ.get('AMD_SERIALIZE_KERNEL', '0')} "
          f"sha256 {h.hexdigest()}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
