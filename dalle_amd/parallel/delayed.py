"""Master-copy optimizer state and the delayed (overlapped) parameter update.

hivemind's ``offload_optimizer=True, delay_optimizer_step=True`` (``task.py:130``, SURVEY §2.6
"Delayed parameter update"): the inner optimizer steps on a separate master copy of the parameters
while the model keeps computing the next micro-batches on the current, one-update-stale parameters;
the new values are copied into the model at a later ``.step()`` call.

MI355X mapping: with 288 GB of HBM the master copy stays on the GPU (one extra fp32 parameter +
gradient arena, 1 GB for the 126M-parameter reference recipe) and the fused LAMB launches run on a
side HIP stream ordered by two events:

  main stream:  ... backward | copy grads+params -> master | (ev_ready) | next fwd/bwd ... | wait(ev_done) | copy master -> model
  side stream:                                  wait(ev_ready) | LAMB grad-norm, moments, trust, apply | (ev_done)

so the optimizer kernels fill the gaps of the next micro-batch's kernels instead of serialising with
them. On CPU peers the same step runs in a background thread (the torch ops release the GIL).

Host offload (``offload_device="cpu"``, the reference's regime: ``CPULAMB8Bit`` on offloaded params,
``lib/training/lamb_8bit.py:138``; and the dead ``lib/training/offload.py`` wrapper's purpose): the
master copy lives in PINNED host memory and the optimizer step runs in the background thread on the
CPU; the pull is one D2H copy of the parameter + gradient arenas, the push one H2D copy. Only for
models whose optimizer state must leave HBM -- with 288 GB per MI355X none of the presets needs it.

Nothing but the master copy is touched by the side stream / thread, and the main stream touches the
master copy only before ``ev_ready`` and after ``ev_done``: the overlap is race-free by
construction.
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional

import torch

from ..optim.flat import FlatArena


class MasterParams:
    """fp32 master copies of the trainable parameters, laid out like the model's arena (identical
    offsets), so model <-> master transfers are single contiguous copies."""

    def __init__(self, params: List[torch.nn.Parameter], arena: Optional[FlatArena] = None, device=None):
        self.model_params = list(params)
        self.model_arena = arena
        order = arena.params if arena is not None else self.model_params
        if arena is not None:
            missing = {id(p) for p in self.model_params} - {id(p) for p in arena.params}
            if missing:
                raise ValueError("every optimised parameter must live in the arena")
        self._of = {}
        masters = []
        for p in order:
            m = torch.nn.Parameter(p.detach().to(device or p.device, dtype=torch.float32, copy=True), requires_grad=True)
            self._of[id(p)] = m
            masters.append(m)
        self.masters = masters
        self.offloaded = bool(masters) and masters[0].device.type == "cpu" and order[0].device.type != "cpu"
        self.arena = FlatArena(masters, device=masters[0].device, pin_memory=self.offloaded) \
            if (arena is not None and masters) else None
        if self.arena is None:
            for m in masters:
                m.grad = torch.zeros_like(m)
        self._pairs = [(p, self._of[id(p)]) for p in order]

    def master_of(self, p: torch.nn.Parameter) -> torch.nn.Parameter:
        return self._of[id(p)]

    def substitute(self, param_groups: List[dict]) -> List[dict]:
        """The optimizer's param groups with every model parameter replaced by its master copy."""
        return [dict(g, params=[self._of[id(p)] for p in g["params"]]) for g in param_groups]

    @torch.no_grad()
    def pull(self):
        """model params + averaged grads -> master (before the step)."""
        if self.arena is not None:
            # D2H for an offloaded master: a synchronous copy -- the host step reads it right after
            self.arena.data.copy_(self.model_arena.data)
            self.arena.grad.copy_(self.model_arena.grad)
            return
        for p, m in self._pairs:
            m.data.copy_(p.data)
            if p.grad is None:
                m.grad.zero_()
            else:
                m.grad.copy_(p.grad)

    @torch.no_grad()
    def push(self):
        """master params -> model (the update becomes visible to compute)."""
        if self.arena is not None:
            self.model_arena.data.copy_(self.arena.data, non_blocking=self.offloaded)  # pinned H2D: async DMA
            return
        for p, m in self._pairs:
            p.data.copy_(m.data)


class AsyncStep:
    """Runs one optimizer update concurrently with the caller's work: on a side HIP stream for GPU
    tensors (event-ordered), in a thread for CPU tensors. At most one update is in flight."""

    def __init__(self, device: torch.device):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self._stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self._done = None
        self._thread: Optional[threading.Thread] = None
        self._error: Optional[BaseException] = None

    @property
    def in_flight(self) -> bool:
        return self._done is not None or self._thread is not None

    def launch(self, fn: Callable[[], None]):
        assert not self.in_flight, "one delayed update at a time"
        if self.cuda:
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self._stream):
                self._stream.wait_event(ready)
                fn()  # enqueues the kernels on the side stream; host-side errors raise here
                self._done = torch.cuda.Event()
                self._done.record(self._stream)
            return

        def run():
            try:
                fn()
            except BaseException as e:  # noqa: BLE001 - re-raised in wait()
                self._error = e

        self._thread = threading.Thread(target=run, name="delayed-optimizer-step", daemon=True)
        self._thread.start()

    def wait(self):
        """Order the caller after the in-flight update (GPU: stream wait, no host sync)."""
        if self.cuda:
            if self._done is not None:
                torch.cuda.current_stream(self.device).wait_event(self._done)
                self._done = None
            return
        if self._thread is not None:
            self._thread.join()
            self._thread = None
            err, self._error = self._error, None
            if err is not None:
                raise err
