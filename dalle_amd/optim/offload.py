"""Optimizer wrappers (reference ``lib/training/wrapper.py:4-47`` and ``lib/training/offload.py:10-93``).

* :class:`OptimizerWrapper` forwards the torch.optim.Optimizer protocol to a wrapped optimizer.
* :class:`OffloadOptimizer` steps on host (CPU) copies of the parameters and gradients and copies the
  result back -- the ZeRO-Offload pattern. On MI355X the fused on-GPU 8-bit LAMB is the default (288 GB
  of HBM leaves no memory reason to offload); offloading remains available for models that do not fit.
"""
from __future__ import annotations

import threading
from typing import Callable, Iterable, Optional

import torch


class OptimizerWrapper(torch.optim.Optimizer):
    def __init__(self, optim: torch.optim.Optimizer):
        self.optim = optim

    def __getstate__(self):
        return self.optim.__getstate__()

    def __setstate__(self, state):
        self.optim.__setstate__(state)

    def __repr__(self):
        return f"{self.__class__.__name__}({repr(self.optim)})"

    @property
    def defaults(self):
        return self.optim.defaults

    @property
    def state(self):
        return self.optim.state

    @property
    def param_groups(self):
        return self.optim.param_groups

    def state_dict(self):
        return self.optim.state_dict()

    def load_state_dict(self, state_dict):
        return self.optim.load_state_dict(state_dict)

    def step(self, *args, **kwargs):
        return self.optim.step(*args, **kwargs)

    def zero_grad(self, *args, **kwargs):
        return self.optim.zero_grad(*args, **kwargs)

    def add_param_group(self, param_group: dict) -> None:
        return self.optim.add_param_group(param_group)


class OffloadOptimizer(OptimizerWrapper):
    """Runs ``optim_cls`` on pinned host copies of the params; ``step()`` copies grads D2H, steps on the
    host and copies the updated params H2D (all under one lock, like the reference)."""

    def __init__(self, param_groups: Iterable, optim_cls: Callable, full_sync: bool = True, offload_device="cpu",
                 offload_dtype: Optional[torch.dtype] = None, **kwargs):
        param_groups = list(param_groups)
        if not isinstance(param_groups[0], dict):
            param_groups = [{"params": param_groups}]
        self.param_groups_main = param_groups
        self.offload_params = []
        host_groups = []
        for group in param_groups:
            hp = []
            for p in group["params"]:
                h = torch.empty_like(p, device=offload_device, dtype=offload_dtype or p.dtype)
                if offload_device == "cpu" and torch.cuda.is_available():
                    h = h.pin_memory()
                h.copy_(p.detach())
                h = torch.nn.Parameter(h, requires_grad=p.requires_grad)
                h.grad = torch.zeros_like(h)
                hp.append(h)
                self.offload_params.append((p, h))
            host_groups.append({**{k: v for k, v in group.items() if k != "params"}, "params": hp})
        super().__init__(optim_cls(host_groups, **kwargs))
        self.full_sync = full_sync
        self.lock = threading.Lock()

    @torch.no_grad()
    def step(self, closure=None, *args, **kwargs):
        assert closure is None, "closure not supported by OffloadOptimizer"
        with self.lock:
            for p, h in self.offload_params:
                if p.grad is not None:
                    h.grad.copy_(p.grad, non_blocking=True)
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            out = self.optim.step(*args, **kwargs)
            for p, h in self.offload_params:
                p.data.copy_(h.data, non_blocking=True)
            return out

    def zero_grad(self, set_to_none: bool = False, *args, **kwargs):
        for p, _ in self.offload_params:
            if p.grad is not None:
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.zero_()
        self.optim.zero_grad(set_to_none=False)
