"""Decentralised (butterfly) all-reduce on RCCL / gloo collectives.

hivemind's AllReduceRunner partitions the flattened vector across peers (client-mode peers get no
shard), every peer reduces its shard from all senders and sends the averaged shard back, with
compression on both legs. On one MI355X node that is exactly

    compress shards -> all_to_all -> dequant + weighted reduce (own shard, fp32) -> compress ->
    all_to_all (reverse splits) -> dequant

so the butterfly maps onto two RCCL all-to-alls over the xGMI mesh (every GPU exchanges 1/N of the
vector with each of its 7 peers at once). Without compression a plain RCCL all-reduce is used.

Averaging is sample-weighted: ``result = sum_p w_p x_p / sum_p w_p``.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from .compression import CompressionBase, NoCompression, SizeAdaptiveCompression


def shard_bounds(numel: int, shard_weights: Sequence[float]) -> List[int]:
    """Split [0, numel) into len(shard_weights) contiguous parts proportional to the weights
    (a zero weight = client-mode peer = empty shard). Identical on every rank."""
    total = float(sum(shard_weights))
    if total <= 0:
        raise ValueError("at least one peer must host a shard")
    bounds = [0]
    acc = 0.0
    for i, w in enumerate(shard_weights):
        acc += w
        bounds.append(numel if i == len(shard_weights) - 1 else int(round(numel * acc / total)))
    return bounds


def _world(group):
    return dist.get_world_size(group), dist.get_rank(group)


def allreduce_weighted(x: torch.Tensor, weight: float, group=None, compression: Optional[CompressionBase] = None,
                       shard_weights: Optional[Sequence[float]] = None, total_weight: Optional[float] = None) -> torch.Tensor:
    """Weighted average of the flat tensor ``x`` across ``group`` (in place when uncompressed).

    ``total_weight`` (sum of the weights) may be given when it is already known (e.g. from the
    progress tracker) to save one collective."""
    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size(group) == 1:
        return x
    W, rank = _world(group)
    if total_weight is None:
        t = torch.tensor([float(weight)], dtype=torch.float64 if x.device.type == "cpu" else torch.float32, device=x.device)
        dist.all_reduce(t, group=group)
        total_weight = float(t.item())
    scale = float(weight) / max(total_weight, 1e-30)
    compression = compression or NoCompression()
    if isinstance(compression, NoCompression):
        x.mul_(scale)
        dist.all_reduce(x, group=group)
        return x
    return butterfly_allreduce(x, scale, group, compression, shard_weights)


def butterfly_allreduce(x: torch.Tensor, scale: float, group, compression: CompressionBase,
                        shard_weights: Optional[Sequence[float]] = None) -> torch.Tensor:
    """Compressed reduce-scatter + all-gather via two all-to-alls. ``x`` is overwritten with the
    average of ``scale_p * x_p`` over peers."""
    W, rank = _world(group)
    flat = x.reshape(-1)
    n = flat.numel()
    shard_weights = list(shard_weights) if shard_weights is not None else [1.0] * W
    b = shard_bounds(n, shard_weights)
    sizes = [b[i + 1] - b[i] for i in range(W)]
    comp = compression.choose(n) if isinstance(compression, SizeAdaptiveCompression) else compression
    contrib = flat.float() * scale

    # ---- leg 1: every shard, compressed, to its owner
    parts = [comp.compress(contrib[b[i]:b[i + 1]]) for i in range(W)]
    keys = sorted(parts[0].keys())
    my = sizes[rank]
    recv = {}
    for k in keys:
        send = torch.cat([p[k].reshape(-1) for p in parts])
        if k == "codebook":
            in_splits = [p[k].numel() for p in parts]
            out_splits = [parts[0][k].numel()] * W
        else:
            in_splits = sizes
            out_splits = [my] * W
        out = torch.empty(sum(out_splits), dtype=send.dtype, device=send.device)
        dist.all_to_all_single(out, send, out_splits, in_splits, group=group)
        recv[k] = (out, out_splits)
    # ---- reduce own shard in fp32
    acc = torch.zeros(my, dtype=torch.float32, device=flat.device)
    offs = {k: 0 for k in keys}
    for src in range(W):
        piece = {}
        for k in keys:
            buf, splits = recv[k]
            piece[k] = buf[offs[k]:offs[k] + splits[src]]
            offs[k] += splits[src]
        if my:
            acc += comp.extract(piece, my)
    # ---- leg 2: averaged shard, compressed, back to everyone
    mine = comp.compress(acc) if my else {k: torch.empty(0, dtype=recv[k][0].dtype, device=flat.device) for k in keys}
    if not my and "codebook" in keys:
        mine["codebook"] = torch.zeros(256, dtype=torch.float32, device=flat.device)
    gathered = {}
    for k in keys:
        send = mine[k].reshape(-1).repeat(W) if mine[k].numel() else mine[k].reshape(-1)
        in_splits = [mine[k].numel()] * W
        if k == "codebook":
            out_splits = [256] * W
        else:
            out_splits = sizes
        out = torch.empty(sum(out_splits), dtype=send.dtype, device=send.device)
        dist.all_to_all_single(out, send, out_splits, in_splits, group=group)
        gathered[k] = (out, out_splits)
    offs = {k: 0 for k in keys}
    for src in range(W):
        piece = {}
        for k in keys:
            buf, splits = gathered[k]
            piece[k] = buf[offs[k]:offs[k] + splits[src]]
            offs[k] += splits[src]
        if sizes[src]:
            flat[b[src]:b[src + 1]] = comp.extract(piece, sizes[src]).to(flat.dtype)
    return x


def broadcast_tensors(tensors: Sequence[torch.Tensor], src: int, group=None):
    """Broadcast a list of tensors from ``src`` (donor) -- used by load_state_from_peers (C3)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    for t in tensors:
        dist.broadcast(t, src=src, group=group)
