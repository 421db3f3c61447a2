"""Learning-rate schedules (``task.py:163-165``: ``get_linear_schedule_with_warmup``)."""
from __future__ import annotations

from torch.optim.lr_scheduler import LambdaLR


def get_linear_schedule_with_warmup(optimizer, num_warmup_steps: int, num_training_steps: int, last_epoch: int = -1):
    """Linear warm-up from 0 to the base lr over ``num_warmup_steps``, then linear decay to 0 at
    ``num_training_steps`` (same curve as transformers' function of that name)."""

    def lr_lambda(current_step: int):
        if current_step < num_warmup_steps:
            return float(current_step) / float(max(1, num_warmup_steps))
        return max(0.0, float(num_training_steps - current_step) / float(max(1, num_training_steps - num_warmup_steps)))

    return LambdaLR(optimizer, lr_lambda, last_epoch)
