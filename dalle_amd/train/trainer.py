"""Collaborative training loop (replaces the HF ``Trainer`` subclass).

Reference behaviour (``lib/training/hf_trainer.py:15-85``, ``run_trainer.py:41-56``):

* micro-batch loop with ``gradient_accumulation_steps`` (loss / accum), then ``optimizer.step()`` on
  the collaborative optimizer and a no-op scheduler (the real scheduler lives in the optimizer);
* ``clip_grad_norm_`` is bypassed (clipping happens inside LAMB on averaged grads);
* ``zero_grad`` is bypassed while all grads are finite when ``reuse_grad_buffers`` (grads keep
  accumulating in ``.grad`` across local steps); non-finite grads are zeroed;
* the data order is seeded per peer (``data_seed``) before the dataloader is built;
* callbacks follow the ``TrainerCallback`` protocol: ``on_train_begin(args, state, control)``,
  ``on_step_end(args, state, control)`` with ``state.log_history[-1]["loss"]`` and
  ``control.should_log``.

No host synchronisation per micro-step: the loss stays a device scalar (``DeferredScalar``: read --
and synced -- only by whoever needs the number, e.g. the callback once per epoch), and the guarded
``zero_grad`` zeroes non-finite accumulated gradients with a device-side flag.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import torch
from torch.utils.data import DataLoader

from ..utils.logging import get_logger
from ..utils.profiling import prof_range

logger = get_logger(__name__)


@dataclass
class TrainerState:
    global_step: int = 0
    epoch: float = 0.0
    log_history: List[Dict[str, Any]] = field(default_factory=list)
    total_flos: float = 0.0


@dataclass
class TrainerControl:
    should_log: bool = False
    should_save: bool = False
    should_training_stop: bool = False


class DeferredScalar:
    """A device scalar that is read lazily: ``float()`` synchronises once and caches the value."""

    __slots__ = ("tensor", "_value")

    def __init__(self, tensor: torch.Tensor):
        self.tensor = tensor.detach()
        self._value = None

    def __float__(self) -> float:
        if self._value is None:
            self._value = float(self.tensor)
        return self._value

    def __repr__(self):
        return f"DeferredScalar({float(self):.6g})"


class TrainerCallback:
    def on_train_begin(self, args, state, control, **kw):
        return control

    def on_step_end(self, args, state, control, **kw):
        return control

    def on_train_end(self, args, state, control, **kw):
        return control


class PrinterCallback(TrainerCallback):
    pass


class ProgressCallback(TrainerCallback):
    pass


class NoOpScheduler(torch.optim.lr_scheduler.LRScheduler):
    """Dummy scheduler for the trainer; the real one is ``collaborative_optimizer.scheduler``."""

    def __init__(self, optimizer):
        self.optimizer = optimizer
        self._last_lr = self.get_lr()

    def get_lr(self):
        return [group["lr"] for group in self.optimizer.param_groups]

    def step(self, *a, **k):
        self._last_lr = self.get_lr()

    def state_dict(self):
        return {}

    def load_state_dict(self, *args, **kwargs):
        pass


class IgnoreGradManipulations(torch.nn.Module):
    """Blocks the loop's zero_grad (while grads are finite) and clip_grad_norm_."""

    def __init__(self, module, override_clipping: bool = True, override_zero_grad: bool = True):
        super().__init__()
        self.module = module
        self.override_clipping = override_clipping
        self.override_zero_grad = override_zero_grad

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def zero_grad(self, set_to_none: bool = False) -> None:
        arena = getattr(self.module, "grad_arena", None)
        if arena is not None:  # one fused finiteness check over the flat gradient arena, on the device
            if self.override_zero_grad:
                from ..ops import zero_grads_if_nonfinite_
                zero_grads_if_nonfinite_(arena.grad)
            else:
                arena.zero_grad()
            return
        params = [p for p in self.parameters() if p.requires_grad and p.grad is not None]
        if self.override_zero_grad and all(torch.isfinite(p.grad).all() for p in params):
            return
        for p in params:
            p.grad.zero_()

    def clip_grad_norm_(self, max_norm: float, norm_type: int = 2):
        if not self.override_clipping:
            return torch.nn.utils.clip_grad_norm_(self.module.parameters(), max_norm, norm_type=norm_type)


class CollaborativeHFTrainer:
    def __init__(self, *, model, args, data_seed: int, collaborative_optimizer, train_dataset=None, data_collator=None,
                 tokenizer=None, eval_dataset=None, callbacks: Optional[List[TrainerCallback]] = None):
        self.args = args
        self.data_seed = int(data_seed) % (2 ** 63)
        self.collaborative_optimizer = collaborative_optimizer
        self.train_dataset, self.data_collator = train_dataset, data_collator
        self.tokenizer = tokenizer
        self.callbacks: List[TrainerCallback] = [PrinterCallback(), ProgressCallback()] + list(callbacks or [])
        self.lr_scheduler = NoOpScheduler(collaborative_optimizer)
        reuse = getattr(getattr(collaborative_optimizer, "grad_averager", None), "reuse_grad_buffers", True)
        self.model = IgnoreGradManipulations(model, override_zero_grad=reuse)
        self.state = TrainerState()
        self.control = TrainerControl()
        self.grad_scaler = None
        if getattr(args, "fp16", False):
            # reference: HivemindGradScaler under --fp16 (D28). The MI355X engine computes in bf16, but the
            # deferred collaborative scaler keeps the flag's semantics (scale, global-step unscale/skip).
            from ..optim.grad_scaler import CollaborativeGradScaler
            self.grad_scaler = CollaborativeGradScaler()
            logger.info("--fp16: loss scaling with the collaborative (global-step deferred) grad scaler")

    def remove_callback(self, cb_type):
        self.callbacks = [c for c in self.callbacks if not (isinstance(c, cb_type) if isinstance(cb_type, type) else c is cb_type)]

    def add_callback(self, cb):
        self.callbacks.append(cb)

    def get_train_dataloader(self) -> DataLoader:
        """Shuffle data independently for each peer to avoid duplicating batches."""
        torch.manual_seed(self.data_seed)
        workers = getattr(self.args, "dataloader_num_workers", 0)
        return DataLoader(self.train_dataset, batch_size=self.args.per_device_train_batch_size, collate_fn=self.data_collator,
                          num_workers=workers, pin_memory=torch.cuda.is_available(),
                          persistent_workers=workers > 0)

    def _call(self, event: str):
        for cb in self.callbacks:
            out = getattr(cb, event)(self.args, self.state, self.control)
            if isinstance(out, TrainerControl):
                self.control = out

    def _device(self):
        return next(self.model.parameters()).device

    def train(self, model_path: Optional[str] = None, resume_from_checkpoint: Optional[str] = None):
        path = resume_from_checkpoint or model_path
        if path is not None:
            ckpt = os.path.join(str(path), "model_state.pt")
            if os.path.isfile(ckpt):
                # The reference called HF train(model_path=...) which required pytorch_model.bin and raised on
                # dirs with only model_state.pt; the task already loaded that file.
                logger.info(f"model weights were restored from {ckpt} by the task")
        args = self.args
        dev = self._device()
        accum = max(1, int(args.gradient_accumulation_steps))
        if hasattr(self.collaborative_optimizer, "set_backwards_per_step"):
            self.collaborative_optimizer.set_backwards_per_step(accum)
        self._call("on_train_begin")
        loader = iter(self.get_train_dataloader())
        max_steps = int(args.max_steps)
        t0 = time.perf_counter()
        while self.state.global_step < max_steps and not self.control.should_training_stop:
            total = None
            for _ in range(accum):
                batch = next(loader)
                batch = {k: v.to(dev, non_blocking=True) for k, v in batch.items()}
                with prof_range("forward"):
                    out = self.model(**batch)
                    loss = out["loss"] / accum
                with prof_range("backward"):
                    (self.grad_scaler.scale(loss) if self.grad_scaler is not None else loss).backward()
                total = loss.detach() if total is None else total + loss.detach()
            self.model.clip_grad_norm_(args.max_grad_norm)
            with prof_range("collaborative_step"):
                if self.grad_scaler is not None:
                    self.grad_scaler.step(self.collaborative_optimizer)
                    self.grad_scaler.update()
                else:
                    self.collaborative_optimizer.step()
            self.lr_scheduler.step()
            self.model.zero_grad()
            self.state.global_step += 1
            self.control.should_log = False
            # the collaborative callback forces should_log every step (callback.py:49): log every step
            self.state.log_history.append({"loss": DeferredScalar(total), "step": self.state.global_step,
                                           "learning_rate": self.collaborative_optimizer.param_groups[0]["lr"],
                                           "elapsed": time.perf_counter() - t0})
            self._call("on_step_end")
        leave = getattr(self.collaborative_optimizer, "leave", None)
        if leave is not None:  # asynchronous peers finish at different times: serve the others' last rounds
            leave()
        apply_pending = getattr(self.collaborative_optimizer, "apply_pending", None)
        if apply_pending is not None:  # a delayed optimizer step still in flight lands in the model
            apply_pending()
        self._call("on_train_end")
        return self.state
