"""Flat parameter / gradient arenas.

All trainable parameters live in ONE contiguous fp32 buffer (and their grads in a second one),
each tensor starting at a 4096-element aligned offset. Consequences on MI355X:

* gradient all-reduce / reduce-scatter runs on large contiguous buckets (no per-tensor launches,
  no copy into a bucket buffer);
* the fused 8-bit LAMB kernel walks the arena with one launch: every 4096-element quantisation
  block belongs to exactly one tensor (the bnb blockwise layout is per tensor);
* grad zeroing, finiteness checks and norms are single kernels.

The ``.data`` / ``.grad`` of every parameter are views into the arenas, so ``state_dict`` and
autograd work unchanged (AccumulateGrad adds into the existing ``.grad`` view in place).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch

ALIGN = 4096


class FlatArena:
    def __init__(self, params: Sequence[torch.nn.Parameter], device=None, dtype=torch.float32, align: int = ALIGN,
                 pin_memory: bool = False):
        seen = set()
        uniq: List[torch.nn.Parameter] = []
        for p in params:
            if id(p) not in seen and p.requires_grad:
                seen.add(id(p))
                uniq.append(p)
        self.params = uniq
        self.align = align
        self.offsets: List[int] = []
        off = 0
        for p in uniq:
            self.offsets.append(off)
            off += (p.numel() + align - 1) // align * align
        self.numel = off
        device = device if device is not None else (uniq[0].device if uniq else "cpu")
        # pinned host arenas (optimizer offload) make the D2H / H2D transfers DMA-able and asynchronous
        pin = bool(pin_memory) and torch.device(device).type == "cpu" and torch.cuda.is_available()
        self.data = torch.zeros(off, dtype=dtype, device=device, pin_memory=pin)
        self.grad = torch.zeros(off, dtype=dtype, device=device, pin_memory=pin)
        for p, o in zip(uniq, self.offsets):
            n = p.numel()
            self.data[o:o + n].copy_(p.data.reshape(-1))
            p.data = self.data[o:o + n].view_as(p)
            p.grad = self.grad[o:o + n].view_as(p)
        self.index: Dict[int, int] = {id(p): i for i, p in enumerate(uniq)}
        # block -> tensor table for the fused kernels (blocks of `align` elements)
        nblocks = off // align
        table = torch.empty(nblocks, dtype=torch.int32)
        for i, (p, o) in enumerate(zip(uniq, self.offsets)):
            b0 = o // align
            b1 = b0 + (p.numel() + align - 1) // align
            table[b0:b1] = i
        self.block_tensor = table.to(device)
        self.sizes = torch.tensor([p.numel() for p in uniq], dtype=torch.int64)
        self.starts = torch.tensor(self.offsets, dtype=torch.int64)

    def zero_grad(self):
        self.grad.zero_()

    def rebind_grads(self):
        """Re-attach ``.grad`` views (after code that set ``p.grad = None``)."""
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            p.grad = self.grad[o:o + n].view_as(p)

    def grads_are_bound(self) -> bool:
        return all(p.grad is not None and p.grad.data_ptr() == self.grad[o:].data_ptr() for p, o in zip(self.params, self.offsets))

    def segments(self) -> List[tuple]:
        """``(offset, numel)`` of every tensor in the flat buffers (the alignment padding excluded):
        the unit the averaging compressors work on (per-tensor choice, per-part codebooks)."""
        return [(o, p.numel()) for p, o in zip(self.params, self.offsets)]

    def tensor_views(self, buf: torch.Tensor) -> List[torch.Tensor]:
        return [buf[o:o + p.numel()].view_as(p) for p, o in zip(self.params, self.offsets)]
