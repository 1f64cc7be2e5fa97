"""Cross-replica BatchNorm (SyncBN) - the reference's ``convert_sync_batchnorm``.

Reference: ``nn.SyncBatchNorm.convert_sync_batchnorm(model, pg)`` (train.py:124),
whose training forward all-gathers ``[mean, invstd, count]`` per layer and whose
backward all-reduces ``[sum_dy, sum_dy_xmu]`` (torch/nn/modules/_functions.py:
39-170).

Here conversion does *not* swap module classes: ``convert_sync_batchnorm``
tags every ``BatchNorm2d`` with ``sync_group`` so parameter names, state_dict
keys and ``isinstance`` checks stay those of plain BN.  The tagged module is
then executed by
* the HIP path (``ops/hip.py``): per-channel partial sums from the conv
  epilogue -> one fp64 exchange of ``[sum, sumsq, count]`` per layer (the
  one-shot xGMI peer kernel ``csrc/peer.hip`` fused with the finalize, or an
  RCCL all-reduce) -> coefficients -> apply; backward exchanges ``[sum dz,
  sum dz*xhat]`` the same way; and
* the reference path below (ATen ops + ``torch.distributed``), which unlike
  torch's SyncBatchNorm also runs on CPU/gloo (used by the W=2 CPU tests).

Statistics are combined with Chan's parallel-variance formula on per-rank
(mean, M2, count) triples, which is exact for unequal per-rank counts.
As in torch, grad_weight/grad_bias are the *local* sums (DDP averages them).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn


def convert_sync_batchnorm(module: nn.Module, group=None) -> nn.Module:
    """Mark every BatchNorm as cross-replica (no-op at world size 1)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return module
    g = group if group is not None else dist.group.WORLD
    for m in module.modules():
        if isinstance(m, nn.modules.batchnorm._BatchNorm):
            m.sync_group = g
    return module


def combine_stats(mean: torch.Tensor, m2: torch.Tensor, count: torch.Tensor):
    """Chan combine of per-rank [W, C] means / M2 with [W] counts -> (mean, biased var, n)."""
    n = count.sum()
    w = (count / n).unsqueeze(1)
    gmean = (mean * w).sum(0)
    d = mean - gmean.unsqueeze(0)
    gm2 = m2.sum(0) + (d * d * count.unsqueeze(1)).sum(0)
    return gmean, gm2 / n, n


class _SyncBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, group):
        dims = [0, 2, 3]
        xf = x.float()
        cnt = xf.numel() // xf.shape[1]
        mean = xf.mean(dims)
        m2 = ((xf - mean.view(1, -1, 1, 1)) ** 2).sum(dims)
        packed = torch.cat([mean, m2, torch.tensor([float(cnt)], device=x.device)])
        from .comm import all_gather_tensor
        allp = all_gather_tensor(packed, group=group)
        c = mean.numel()
        gmean, gvar, n = combine_stats(allp[:, :c], allp[:, c:2 * c], allp[:, 2 * c])
        invstd = torch.rsqrt(gvar + eps)
        if running_mean is not None:
            with torch.no_grad():
                unbiased = gvar * (n / (n - 1).clamp(min=1))
                running_mean.mul_(1 - momentum).add_(gmean * momentum)
                running_var.mul_(1 - momentum).add_(unbiased * momentum)
        ctx.save_for_backward(x, weight, gmean, invstd)
        ctx.group, ctx.n = group, n
        y = (xf - gmean.view(1, -1, 1, 1)) * (invstd * weight).view(1, -1, 1, 1) + bias.view(1, -1, 1, 1)
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        x, weight, mean, invstd = ctx.saved_tensors
        dims = [0, 2, 3]
        dyf = dy.float()
        xhat = (x.float() - mean.view(1, -1, 1, 1)) * invstd.view(1, -1, 1, 1)
        sum_dy = dyf.sum(dims)
        sum_dy_xhat = (dyf * xhat).sum(dims)
        gw, gb = sum_dy_xhat.clone(), sum_dy.clone()  # local, as torch SyncBN
        red = torch.cat([sum_dy, sum_dy_xhat])
        dist.all_reduce(red, group=ctx.group)
        c = sum_dy.numel()
        mdy = (red[:c] / ctx.n).view(1, -1, 1, 1)
        mdyx = (red[c:] / ctx.n).view(1, -1, 1, 1)
        dx = (dyf - mdy - xhat * mdyx) * (invstd * weight).view(1, -1, 1, 1)
        return dx.to(dy.dtype), gw, gb, None, None, None, None, None


def sync_batch_norm(x: torch.Tensor, bn: nn.BatchNorm2d, group) -> torch.Tensor:
    if bn.training and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    mom = bn.momentum if bn.momentum is not None else 0.1
    return _SyncBN.apply(x, bn.weight, bn.bias, bn.running_mean if bn.track_running_stats else None,
                         bn.running_var if bn.track_running_stats else None, bn.eps, mom, group)
