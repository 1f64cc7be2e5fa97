"""Adam with a fused multi-tensor HIP kernel, plus the reference's MultiStepLR.

Reference: ``Adam(model.parameters(), lr=0.5e-5)`` (train.py:126-127; defaults
betas (0.9, 0.999), eps 1e-8, weight_decay 0) and
``MultiStepLR(optimizer, milestones=[50, 80], gamma=0.5)`` (train.py:156).

GPU path: ONE kernel launch per step updates every parameter: it reads fp32
param / grad / m / v, applies the gradient scale (the reducer's 1/world mean),
writes fp32 param / m / v and the bf16 weight *shadow* that the conv kernels
consume - the cast is fused, there is no separate bf16 conversion pass.  The
step count and learning rate live in device memory so the launch is HIP-graph
capturable.  CPU path: the same math with ATen ops.

``state_dict`` uses torch.optim.Adam's format (per-param ``step``, ``exp_avg``,
``exp_avg_sq``), so checkpoints interoperate with stock Adam.
"""
from __future__ import annotations

import math

import torch
from torch.optim import Optimizer
from torch.optim.lr_scheduler import MultiStepLR  # noqa: F401  (re-export)


class FusedAdam(Optimizer):
    def __init__(self, params, lr=0.5e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._table = None
        self._table_key = None
        self._dev_scalars = None

    # -------------------------------------------------------------- state
    def _sync_host_steps(self):
        """Copy the device-side step counters into ``state[p]['step']`` (checkpoint time only)."""
        for gi, t in getattr(self, "_lr_step", {}).items():
            step = float(t[1].item())
            for p in self.param_groups[gi]["params"]:
                if p in self.state and "step" in self.state[p]:
                    self.state[p]["step"] = torch.tensor(step, dtype=torch.float32)

    def state_dict(self):
        self._sync_host_steps()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        for st in self.state.values():
            if "step" in st and isinstance(st["step"], torch.Tensor):
                st["step"] = st["step"].detach().to("cpu", torch.float32)
        self._lr_step = {}
        self._table = None
        self._table_key = None

    # -------------------------------------------------------------- helpers
    def _params_with_grad(self):
        for gi, group in enumerate(self.param_groups):
            for p in group["params"]:
                if p.grad is not None:
                    yield gi, group, p

    def _init_state(self, p):
        st = self.state[p]
        if len(st) == 0:
            st["step"] = torch.zeros((), dtype=torch.float32)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        return st

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = closure() if closure is not None else None
        items = list(self._params_with_grad())
        if not items:
            return loss
        if items[0][2].is_cuda:
            from ..ops import functional as Fx
            if Fx.get_backend() != "torch":
                self._step_hip(items, grad_scale)
                return loss
        self._step_ref(items, grad_scale)
        return loss

    def _step_ref(self, items, grad_scale):
        for _gi, group, p in items:
            st = self._init_state(p)
            b1, b2 = group["betas"]
            st["step"] += 1
            t = float(st["step"])
            g = p.grad if grad_scale == 1.0 else p.grad * grad_scale
            if group["weight_decay"]:
                g = g.add(p, alpha=group["weight_decay"])
            st["exp_avg"].mul_(b1).add_(g, alpha=1 - b1)
            st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
            bc1 = 1 - b1 ** t
            bc2 = 1 - b2 ** t
            denom = (st["exp_avg_sq"].sqrt() / math.sqrt(bc2)).add_(group["eps"])
            p.addcdiv_(st["exp_avg"], denom, value=-group["lr"] / bc1)

    def _step_hip(self, items, grad_scale):
        from ..ops import hip
        for _gi, _group, p in items:
            self._init_state(p)
        key = (hip.shadow_generation(),) + tuple((p.data_ptr(), p.grad.data_ptr()) for _gi, _g, p in items)
        if key != self._table_key:
            self._table = hip.adam_build_table(self, items)
            self._table_key = key
        hip.adam_step(self, items, self._table, grad_scale)
