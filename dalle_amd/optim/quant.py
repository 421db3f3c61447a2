"""Blockwise 8-bit quantisation with the bitsandbytes dynamic maps.

``lib/training/lamb_8bit.py:79-81,115-117`` fills ``qmap1 = dynamic(signed)`` and
``qmap2 = udynamic(unsigned)``; moments are stored per 4096-element block as the index of the
nearest map entry of ``x / absmax(block)``. Dequantisation is ``code[q] * absmax[block]``.

This module holds the maps (bit-exact re-derivation of ``create_dynamic_map``) and a vectorised
PyTorch implementation used on CPU and as the numerics golden of the HIP kernels
(``csrc/optim/lamb8bit.hip``).
"""
from __future__ import annotations

from functools import lru_cache

import torch

BLOCK = 4096


@lru_cache(maxsize=4)
def _dynamic_map_cpu(signed: bool = True, n: int = 7) -> torch.Tensor:
    data = []
    additional_items = 2 ** (7 - n) - 1
    if not signed:
        additional_items = 2 * additional_items
    for i in range(n):
        fraction_items = 2 ** (i + 7 - n) + 1 if signed else 2 ** (i + 7 - n + 1) + 1
        boundaries = torch.linspace(0.1, 1, fraction_items)
        means = (boundaries[:-1] + boundaries[1:]) / 2.0
        data += ((10 ** (-(n - 1) + i)) * means).tolist()
        if signed:
            data += (-(10 ** (-(n - 1) + i)) * means).tolist()
    if additional_items > 0:
        boundaries = torch.linspace(0.1, 1, additional_items + 1)
        means = (boundaries[:-1] + boundaries[1:]) / 2.0
        data += ((10 ** (-(n - 1) + i)) * means).tolist()
        if signed:
            data += (-(10 ** (-(n - 1) + i)) * means).tolist()
    data.append(0)
    data.append(1.0)
    data.sort()
    return torch.tensor(data, dtype=torch.float32)


def dynamic_map(signed: bool = True, device=None) -> torch.Tensor:
    m = _dynamic_map_cpu(signed).clone()
    return m.to(device) if device is not None else m


def num_blocks(n: int, block: int = BLOCK) -> int:
    return (n + block - 1) // block


def quantize_blockwise(x: torch.Tensor, code: torch.Tensor, block: int = BLOCK):
    """Returns (uint8 indices shaped like x, absmax (num_blocks,) fp32). Nearest-entry rounding."""
    flat = x.reshape(-1).float()
    n = flat.numel()
    nb = num_blocks(n, block)
    pad = nb * block - n
    xb = torch.nn.functional.pad(flat, (0, pad)).view(nb, block)
    absmax = xb.abs().amax(dim=1)
    normed = xb / absmax.clamp(min=1e-30)[:, None]
    code = code.to(x.device).float()
    # nearest code entry via searchsorted on the sorted map + neighbour compare
    idx = torch.searchsorted(code, normed.contiguous()).clamp(1, code.numel() - 1)
    lo, hi = code[idx - 1], code[idx]
    q = torch.where((normed - lo).abs() <= (hi - normed).abs(), idx - 1, idx)
    q = q.view(-1)[:n].to(torch.uint8).view_as(x)
    return q, absmax


def dequantize_blockwise(q: torch.Tensor, absmax: torch.Tensor, code: torch.Tensor, block: int = BLOCK) -> torch.Tensor:
    flat = q.reshape(-1).long()
    n = flat.numel()
    vals = code.to(q.device).float()[flat]
    scale = absmax.repeat_interleave(block)[:n]
    return (vals * scale).view(q.shape)
