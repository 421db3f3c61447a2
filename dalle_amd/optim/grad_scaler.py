"""Loss scaler for collaborative training (counterpart of hivemind's ``GradScaler`` used by the
reference when ``--fp16 True``; SURVEY D28, ``arguments.py:29``).

A plain AMP scaler unscales, checks for inf/NaN and updates its scale after EVERY local step. In
collaborative training the gradients of many local steps accumulate (scaled) in ``.grad`` and are
only consumed at the global step, so this scaler defers all three to that moment:

* ``scale(loss)``                 -- multiply the loss by the current scale (every micro-step);
* ``step(optimizer)``             -- forwards to ``CollaborativeOptimizer.step(grad_scaler=self)``;
  when the collaboration is ready for a global step, the optimizer calls ``unscale_and_check``
  on the accumulated grads before averaging and skips the update if any peer saw inf/NaN;
* ``update()``                    -- adjusts the scale ONLY after a global step (grow after
  ``growth_interval`` clean global steps, back off on overflow), so local steps never change the
  scale that grads already accumulated under.

The MI355X engine computes in bf16, whose exponent range makes loss scaling unnecessary; the
scaler is kept for checkpoint/CLI compatibility and for fp16 experiments on the reference path.
"""
from __future__ import annotations

from typing import Iterable, Optional

import torch
import torch.distributed as dist


class CollaborativeGradScaler:
    def __init__(self, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0, backoff_factor: float = 0.5,
                 growth_interval: int = 2000, enabled: bool = True):
        self._scale = float(init_scale)
        self.growth_factor, self.backoff_factor = float(growth_factor), float(backoff_factor)
        self.growth_interval = int(growth_interval)
        self._growth_tracker = 0
        self._enabled = bool(enabled)
        self._pending_global: Optional[bool] = None  # None: no global step since last update(); else found_inf

    # -- torch.amp.GradScaler-compatible surface ---------------------------------------------------
    def is_enabled(self) -> bool:
        return self._enabled

    def get_scale(self) -> float:
        return self._scale if self._enabled else 1.0

    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        return loss * self._scale if self._enabled else loss

    def step(self, optimizer, *args, **kwargs):
        """Local step: hand the scaler to the collaborative optimizer (which unscales only at the global
        step). For a plain torch optimizer, behave like a regular AMP scaler."""
        if not self._enabled:
            return optimizer.step(*args, **kwargs)
        if hasattr(optimizer, "grad_averager"):
            return optimizer.step(*args, grad_scaler=self, **kwargs)
        grads = [p.grad for g in optimizer.param_groups for p in g["params"] if p.grad is not None]
        if self.unscale_and_check(grads):
            optimizer.step(*args, **kwargs)
        return None

    def unscale_(self, optimizer):
        """Deferred: unscaling happens once per GLOBAL step inside ``unscale_and_check``."""
        return None

    def update(self, new_scale: Optional[float] = None):
        if not self._enabled:
            return
        if new_scale is not None:
            self._scale = float(new_scale)
            self._pending_global = None
            return
        if self._pending_global is None:  # no global step happened: the scale must stay put
            return
        if self._pending_global:
            self._scale *= self.backoff_factor
            self._growth_tracker = 0
        else:
            self._growth_tracker += 1
            if self._growth_tracker >= self.growth_interval:
                self._scale *= self.growth_factor
                self._growth_tracker = 0
        self._pending_global = None

    # -- called by CollaborativeOptimizer at the global step ------------------------------------------
    @torch.no_grad()
    def unscale_and_check(self, grads: Iterable[torch.Tensor] = (), flat_grad: Optional[torch.Tensor] = None,
                          group=None, local_only: bool = False) -> bool:
        """Unscale the accumulated grads in place and return True if they are finite on EVERY rank of
        ``group`` (one tiny all-reduce), False otherwise (the caller then skips the update).
        ``local_only``: check this rank's grads only, with no collective -- for a round whose
        communicator just failed (a collective queued behind the broken one would hang the peer)."""
        inv = 1.0 / self._scale
        bufs = [flat_grad] if flat_grad is not None else [g for g in grads if g is not None]
        bad = None
        for b in bufs:
            b.mul_(inv)
            nb = (~torch.isfinite(b)).any()
            bad = nb if bad is None else (bad | nb)
        flag = torch.zeros((), dtype=torch.float32, device=bufs[0].device if bufs else "cpu")
        if bad is not None:
            flag = bad.float()
        if not local_only and dist.is_available() and dist.is_initialized():
            world = dist.get_world_size(group) if group is not None else dist.get_world_size()
            if world > 1:
                flag = flag.reshape(1)
                dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        found_inf = bool(flag.item() > 0)
        self._pending_global = found_inf
        return not found_inf

    # -- checkpointing ------------------------------------------------------------------------------
    def state_dict(self) -> dict:
        return {"scale": self._scale, "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval, "_growth_tracker": self._growth_tracker}

    def load_state_dict(self, sd: dict):
        self._scale = float(sd["scale"])
        self.growth_factor = float(sd.get("growth_factor", self.growth_factor))
        self.backoff_factor = float(sd.get("backoff_factor", self.backoff_factor))
        self.growth_interval = int(sd.get("growth_interval", self.growth_interval))
        self._growth_tracker = int(sd.get("_growth_tracker", 0))


# hivemind name
GradScaler = CollaborativeGradScaler
