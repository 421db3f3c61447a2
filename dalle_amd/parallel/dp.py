"""Data-parallel gradient synchronisation over RCCL (xGMI) / gloo.

The gradient arena is one contiguous buffer (``FlatArena``), so a bucket is just a slice: no pack /
unpack copies. Buckets are sized for the xGMI mesh: each of the 8 GPUs has 7
point-to-point links; RCCL splits an all-reduce into per-peer slices, and a 64 MB bucket keeps each
per-link slice at >= 4 MB, past the latency-bound regime, while still pipelining several
collectives. With weight sharing (5 blocks reused by every layer, tied embedding) no gradient is
final before the end of backward, so all buckets are issued after ``backward()``: RCCL runs them on
its own stream back to back, and the compute stream only waits for them (``Work.wait`` is a stream
dependency, not a host block) before the optimizer kernels -- nothing overlaps the all-reduce itself.

``grad_dtype='bf16'`` halves the bytes on the wire (the averaged gradient is accumulated in fp32
by RCCL's reduction of bf16 inputs is bf16 -- use for large worlds only).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..optim.flat import FlatArena

DEFAULT_BUCKET_BYTES = 64 * 1024 * 1024


class GradSync:
    def __init__(self, arena: FlatArena, world_size: int = 1, group=None, grad_dtype: str = "fp32",
                 bucket_bytes: int = DEFAULT_BUCKET_BYTES, average: bool = True):
        self.arena = arena
        self.world_size = world_size
        self.group = group
        self.grad_dtype = grad_dtype
        self.average = average
        elems = max(1, bucket_bytes // 4)
        self.buckets = [(s, min(s + elems, arena.numel)) for s in range(0, arena.numel, elems)]
        self._lowp = None

    @torch.no_grad()
    def all_reduce(self):
        if self.world_size <= 1:
            return
        g = self.arena.grad
        if self.grad_dtype == "bf16":
            if self._lowp is None:
                self._lowp = torch.empty(g.numel(), dtype=torch.bfloat16, device=g.device)
            lp = self._lowp
            lp.copy_(g)
            works = [dist.all_reduce(lp[s:e], group=self.group, async_op=True) for s, e in self.buckets]
            for w in works:
                w.wait()
            g.copy_(lp)
        else:
            works = [dist.all_reduce(g[s:e], group=self.group, async_op=True) for s, e in self.buckets]
            for w in works:
                w.wait()
        if self.average:
            g.mul_(1.0 / self.world_size)
