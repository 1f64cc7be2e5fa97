"""Metrics: ``AverageMeter`` / ``Accuracy`` (reference utils.py:5-27) plus
device-side accumulators that avoid the per-step / per-sample host syncs of the
reference (train.py:64-68, 88-90; defects A14, A21)."""
from __future__ import annotations

import torch


class AverageMeter:
    """Computes and stores the average and current value (reference utils.py:5-20)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val = 0
        self.avg = 0
        self.sum = 0
        self.count = 0

    def update(self, val, n=1):
        self.val = val
        self.sum += val * n
        self.count += n
        self.avg = self.sum / self.count


def Accuracy(out, label):  # noqa: N802  (reference name)
    """1 where argmax(out, 1) == label (reference utils.py:25-27)."""
    _, pred = torch.max(out, dim=1)
    return 1 * (pred == label)


class DeviceMeter:
    """Loss meter that stays on device: ``update`` launches no host sync.

    ``val``/``avg`` sync only when read (e.g. at log interval).
    """

    def __init__(self, device):
        self.sum = torch.zeros((), dtype=torch.float64, device=device)
        self.count = 0
        self.last = torch.zeros((), dtype=torch.float32, device=device)

    def update(self, val: torch.Tensor, n: int = 1):
        self.last.copy_(val.detach())
        self.sum.add_(val.detach().double() * n)
        self.count += n

    @property
    def val(self) -> float:
        return float(self.last)

    @property
    def avg(self) -> float:
        return float(self.sum) / max(self.count, 1)


class AccuracyCounter:
    """Top-1 correct/total counters kept on device (validation without per-sample ``.cpu()``)."""

    def __init__(self, device):
        self.correct = torch.zeros((), dtype=torch.int64, device=device)
        self.total = torch.zeros((), dtype=torch.int64, device=device)

    @torch.no_grad()
    def update(self, logits: torch.Tensor, labels: torch.Tensor, valid: torch.Tensor | None = None):
        hit = (logits.argmax(1) == labels)
        if valid is not None:
            hit = hit & valid
            self.total += valid.sum()
        else:
            self.total += labels.numel()
        self.correct += hit.sum()
