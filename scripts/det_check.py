"""Is a --deterministic HIP training run bitwise reproducible?  Trains MODEL twice from the same seed (the
tests/test_gpu_learning.py setup, HIP side only) and reports the first step whose loss differs.
    python scripts/det_check.py [model] [size] [steps] [batch]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

from test_gpu_learning import _data, _run  # noqa: E402

model = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
size = int(sys.argv[2]) if len(sys.argv) > 2 else 96
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 40
batch = int(sys.argv[4]) if len(sys.argv) > 4 else 32
train = _data(max(steps * batch // 3, 4 * batch), size, seed=11)
val = _data(64, size, seed=12)
a, _ = _run(model, size, "hip", "bf16", steps, batch, 1e-3, train, val, det=True)
b, _ = _run(model, size, "hip", "bf16", steps, batch, 1e-3, train, val, det=True)
diff = (a != b).nonzero()
first = int(diff[0]) if diff.numel() else -1
print(f"{model}: bitwise equal={bool(torch.equal(a, b))} first differing step={first} "
      f"loss[0]={a[0].item():.6f}/{b[0].item():.6f} loss[-1]={a[-1].item():.4f}/{b[-1].item():.4f}")
