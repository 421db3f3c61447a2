"""Tensor compression for collaborative averaging (``task.py:125-126``).

``SizeAdaptiveCompression(threshold=2**16+1, less=Float16Compression(), greater_equal=Uniform8BitQuantization())``
is the reference's choice for both gradient and state averaging.

* ``Float16Compression``: clamp to the fp16 range and cast (2 B/elem).
* ``Uniform8BitQuantization``: centre by the mean, ``scale = 6 sigma / 256``, ``q = clamp(round(x/scale)
  + 128, 0, 255)``; the codebook is the **per-bin mean** of the original values (256 floats), and
  dequantisation is ``codebook[q]`` (1 B/elem + 1 KiB).
* ``NoCompression``.

All compressors work on device tensors (HIP on MI355X): a compressed tensor is a small dict of
tensors so it can ride RCCL all-to-all / all-gather directly (see ``averaging.py``).
"""
from __future__ import annotations

import math
from typing import Dict

import torch

Compressed = Dict[str, torch.Tensor]


class CompressionBase:
    name = "base"

    def compress(self, x: torch.Tensor) -> Compressed:
        raise NotImplementedError

    def extract(self, c: Compressed, numel: int) -> torch.Tensor:
        raise NotImplementedError

    def roundtrip(self, x: torch.Tensor) -> torch.Tensor:
        return self.extract(self.compress(x), x.numel()).view_as(x)

    def bytes_per_element(self) -> float:
        return 4.0


class NoCompression(CompressionBase):
    name = "none"

    def compress(self, x):
        return {"data": x.reshape(-1).float()}

    def extract(self, c, numel):
        return c["data"].float()


class Float16Compression(CompressionBase):
    name = "fp16"
    FP16_MAX = 65504.0

    def compress(self, x):
        return {"data": x.reshape(-1).float().clamp(-self.FP16_MAX, self.FP16_MAX).to(torch.float16)}

    def extract(self, c, numel):
        return c["data"].float()

    def bytes_per_element(self):
        return 2.0


def average_buckets(values: torch.Tensor, indices: torch.Tensor, n_bins: int) -> torch.Tensor:
    """Per-bin mean of ``values`` (the 8-bit codebook)."""
    idx = indices.reshape(-1).long()
    sums = torch.zeros(n_bins, dtype=torch.float32, device=values.device).scatter_add_(0, idx, values.reshape(-1).float())
    counts = torch.zeros(n_bins, dtype=torch.float32, device=values.device).scatter_add_(0, idx, torch.ones_like(idx, dtype=torch.float32))
    return sums / counts.clamp_min(1)


class Uniform8BitQuantization(CompressionBase):
    name = "uniform8bit"
    RANGE_IN_SIGMAS = 6
    n_bins = 256

    def compress(self, x):
        x = x.reshape(-1).float()
        if x.is_cuda:
            # fused HIP passes with an integer (deterministic) codebook reduction: csrc/kernels/quant.hip
            from ..ops.ext import load_extension

            q, cb = load_extension(required=True).uq8_compress(x.contiguous())
            return {"idx": q, "codebook": cb}
        n = x.numel()
        shift = x.mean()
        centered = x - shift
        std = centered.norm() / math.sqrt(max(n - 1, 1))
        scale = (self.RANGE_IN_SIGMAS * std / self.n_bins).clamp_min(1e-30)
        q = torch.clamp(torch.round(centered / scale) + self.n_bins // 2, 0, self.n_bins - 1).to(torch.uint8)
        return {"idx": q, "codebook": average_buckets(x, q, self.n_bins)}

    def extract(self, c, numel):
        if c["idx"].is_cuda:
            from ..ops.ext import load_extension

            out = torch.empty(c["idx"].numel(), dtype=torch.float32, device=c["idx"].device)
            load_extension(required=True).uq8_dequant_(c["idx"].contiguous(), c["codebook"].float().contiguous(), out, 1.0, False)
            return out
        return c["codebook"][c["idx"].long()]

    def bytes_per_element(self):
        return 1.0


class SizeAdaptiveCompression(CompressionBase):
    """``less`` for tensors with fewer than ``threshold`` elements, ``greater_equal`` otherwise."""

    name = "size_adaptive"

    def __init__(self, threshold: int, less: CompressionBase, greater_equal: CompressionBase):
        self.threshold, self.less, self.greater_equal = threshold, less, greater_equal

    def choose(self, numel: int) -> CompressionBase:
        return self.less if numel < self.threshold else self.greater_equal

    def compress(self, x):
        return self.choose(x.numel()).compress(x)

    def extract(self, c, numel):
        return self.choose(numel).extract(c, numel)


def reference_averaging_compression() -> SizeAdaptiveCompression:
    """The reference's gradient / state averaging compression (``task.py:125-126``)."""
    return SizeAdaptiveCompression(threshold=2 ** 16 + 1, less=Float16Compression(), greater_equal=Uniform8BitQuantization())
