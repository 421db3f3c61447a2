"""Reversible residual engine (``reversible=True`` at ``task.py:81``).

Coupling on a duplicated stream: ``x -> [x, x]``; per block ``y1 = x1 + f(x2)``,
``y2 = x2 + g(y1)``; the stack output is the mean of the two halves. Activations are not stored:
the backward pass reconstructs every block input from its output and recomputes ``f``/``g`` (with
the fused HIP kernels) to get the gradients -- O(1) activation memory in depth.

Dropout is compile-time off in every recipe we support, so there is no RNG state to replay
(the reference's ``Deterministic`` wrapper survives only as a state-dict naming level).
Shared modules simply accumulate their gradients across the blocks that reuse them.
"""
from __future__ import annotations

from typing import Callable, List, Sequence, Tuple

import torch

Branch = Callable[[torch.Tensor], torch.Tensor]


class _ReversibleFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x1, x2, fns: Sequence[Tuple[Branch, Branch]]):
        ctx.fns = fns
        with torch.no_grad():
            for f, g in fns:
                x1 = x1 + f(x2)
                x2 = x2 + g(x1)
        y1, y2 = x1.detach(), x2.detach()
        ctx.save_for_backward(y1, y2)
        return y1, y2

    @staticmethod
    def backward(ctx, dy1, dy2):
        y1, y2 = ctx.saved_tensors
        fns = ctx.fns
        for f, g in reversed(fns):
            # reconstruct x2 = y2 - g(y1) and get grads through g
            with torch.enable_grad():
                y1r = y1.detach().requires_grad_(True)
                gy1 = g(y1r)
                torch.autograd.backward(gy1, dy2)
            with torch.no_grad():
                x2 = y2 - gy1
                dy1 = dy1 + y1r.grad
                del gy1, y1r
            # reconstruct x1 = y1 - f(x2) and get grads through f
            with torch.enable_grad():
                x2r = x2.detach().requires_grad_(True)
                fx2 = f(x2r)
                torch.autograd.backward(fx2, dy1)
            with torch.no_grad():
                x1 = y1 - fx2
                dy2 = dy2 + x2r.grad
                del fx2, x2r
            y1, y2 = x1, x2
        return dy1, dy2, None


def reversible_sequence(x: torch.Tensor, fns: List[Tuple[Branch, Branch]]) -> torch.Tensor:
    """Run the reversible stack on ``[x, x]`` and return the mean of the two output halves."""
    y1, y2 = _ReversibleFunction.apply(x, x, fns)
    return (y1 + y2) * 0.5
