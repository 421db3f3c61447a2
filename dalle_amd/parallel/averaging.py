"""Decentralised (butterfly) all-reduce on RCCL / gloo collectives.

hivemind's AllReduceRunner partitions the flattened tensors across peers (client-mode peers get no
shard). Every peer reduces its shard from all senders and sends the averaged shard back, and every
PART of every TENSOR is compressed on its own: the compressor is picked from the size of the whole
tensor (``SizeAdaptiveCompression``: fp16 below 2^16+1 elements, uniform 8-bit above) and an 8-bit
part carries its own 256-entry codebook. On one MI355X node the butterfly is two legs of RCCL
collectives over the xGMI mesh:

    leg 1: compress every (tensor, shard) part -> all_to_all (each GPU sends 1/N to each of its 7 peers)
           -> dequantise + weighted fp32 reduce of the own shard
    leg 2: compress the averaged shard -> all_gather -> dequantise into place

Which element goes where in which format is a pure function of (numel, tensor segments, shard
weights, compressor), computed once per averager as a :class:`ButterflyPlan` with its device-side
part tables, so a round costs a handful of launches: ONE segmented quantise launch for all 8-bit
parts of a leg (``csrc/kernels/quant.hip``: one workgroup per part), one gather + cast for all
elementwise (fp16 / fp32) parts, and one segmented dequantise launch per source peer.

Without compression a plain RCCL all-reduce is used. Averaging is sample-weighted:
``result = sum_p w_p x_p / sum_p w_p``.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .compression import (CompressionBase, Float16Compression, NoCompression, SizeAdaptiveCompression,
                          Uniform8BitQuantization)

# hivemind streams tensors in parts of 2^19 bytes of the uncompressed fp32 tensor; each part is
# compressed separately (one codebook per part for the 8-bit quantiser)
PART_ELEMS = 2 ** 17


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


def _codec(comp: CompressionBase) -> str:
    if isinstance(comp, Uniform8BitQuantization):
        return "u8"
    if isinstance(comp, Float16Compression):
        return "fp16"
    if isinstance(comp, NoCompression):
        return "fp32"
    raise TypeError(f"butterfly: unsupported compressor {type(comp).__name__}")


class ButterflyPlan:
    """Per-owner element sets of one butterfly round.

    * elementwise parts (fp16 / fp32 codecs): ``e_idx[d]`` = flat positions owned by peer ``d``;
    * 8-bit parts: ``(flat_offset, length)`` pieces of at most ``part_elems`` elements, each inside one
      tensor and one shard, with their packed offsets in the owner's 8-bit payload.
    """

    def __init__(self, numel: int, segments: Sequence[Tuple[int, int]], shard_weights: Sequence[float],
                 compression: CompressionBase, device, part_elems: int = PART_ELEMS):
        W = len(shard_weights)
        b = shard_bounds(numel, shard_weights)
        self.W, self.bounds, self.device = W, b, torch.device(device)
        e_dtype = None
        e_pos: List[List[torch.Tensor]] = [[] for _ in range(W)]
        u_parts: List[List[Tuple[int, int]]] = [[] for _ in range(W)]
        for off, n in segments:
            if n <= 0:
                continue
            comp = compression.choose(n) if isinstance(compression, SizeAdaptiveCompression) else compression
            codec = _codec(comp)
            for d in range(W):
                lo, hi = max(off, b[d]), min(off + n, b[d + 1])
                if lo >= hi:
                    continue
                if codec == "u8":
                    for s in range(lo, hi, part_elems):
                        u_parts[d].append((s, min(part_elems, hi - s)))
                else:
                    dt = torch.float16 if codec == "fp16" else torch.float32
                    if e_dtype is not None and e_dtype != dt:
                        raise ValueError("butterfly: at most one elementwise codec per round")
                    e_dtype = dt
                    e_pos[d].append(torch.arange(lo, hi, dtype=torch.int64))
        self.e_dtype = e_dtype or torch.float16
        self.e_idx = [torch.cat(p) if p else torch.zeros(0, dtype=torch.int64) for p in e_pos]
        self.e_sizes = [int(t.numel()) for t in self.e_idx]
        self.e_idx_all = torch.cat(self.e_idx).to(self.device)
        self.e_idx_dev = [t.to(self.device) for t in self.e_idx]
        self.u_parts = u_parts
        self.u_sizes = [sum(n for _, n in ps) for ps in u_parts]   # 8-bit elements per owner
        self.p_counts = [len(ps) for ps in u_parts]                # 8-bit parts per owner
        # leg-1 compression tables over ALL parts (owner-major), packed offsets into the send payload
        flat_off, packed_off, lens = [], [], []
        acc = 0
        self.owner_packed_start = []
        for d in range(W):
            self.owner_packed_start.append(acc)
            for s, n in u_parts[d]:
                flat_off.append(s)
                packed_off.append(acc)
                lens.append(n)
                acc += n
        self.u_total = acc
        self.flat_end = max((s + n for ps in u_parts for s, n in ps), default=0)
        self.own_flat_end = [max((s + n for s, n in ps), default=0) for ps in u_parts]
        self.t_flat_off = torch.tensor(flat_off, dtype=torch.int64, device=self.device)
        self.t_packed_off = torch.tensor(packed_off, dtype=torch.int64, device=self.device)
        self.t_len = torch.tensor(lens, dtype=torch.int32, device=self.device)
        # per owner: offsets relative to that owner's own payload, and flat offsets (leg 2 / extraction)
        self.own_rel_off, self.own_flat_off, self.own_len = [], [], []
        for d in range(W):
            rel, fl, ln = [], [], []
            acc = 0
            for s, n in u_parts[d]:
                rel.append(acc)
                fl.append(s)
                ln.append(n)
                acc += n
            self.own_rel_off.append(torch.tensor(rel, dtype=torch.int64, device=self.device))
            self.own_flat_off.append(torch.tensor(fl, dtype=torch.int64, device=self.device))
            self.own_len.append(torch.tensor(ln, dtype=torch.int32, device=self.device))
        self.numel = numel

    def wire_bytes(self) -> int:
        """Bytes one peer sends in leg 1 (a full copy of the vector, compressed)."""
        esz = torch.finfo(self.e_dtype).bits // 8
        return sum(self.e_sizes) * esz + self.u_total + sum(self.p_counts) * 256 * 4


_PLANS: "OrderedDict[tuple, ButterflyPlan]" = OrderedDict()


def get_plan(numel, segments, shard_weights, compression, device) -> ButterflyPlan:
    key = (numel, tuple(map(tuple, segments)), tuple(float(w) for w in shard_weights), id(compression), str(device))
    plan = _PLANS.get(key)
    if plan is None:
        plan = ButterflyPlan(numel, segments, shard_weights, compression, device)
        _PLANS[key] = plan
        while len(_PLANS) > 8:
            _PLANS.popitem(last=False)
    return plan


# ---- segmented 8-bit codec: HIP kernels on the GPU, per-part torch on CPU peers -----------------
def _seg_compress(x, x_off, q_off, lens, q, cb, x_end: int, q_end: int):
    """Quantise parts ``x[x_off[i]:+len[i]]`` into ``q[q_off[i]:+len[i]]`` + ``cb[256 i:+256]``.
    ``x_end`` / ``q_end``: host-known extents of the part tables (checked against the buffers)."""
    if not lens.numel():
        return
    if x.is_cuda:
        from ..ops.ext import load_extension
        load_extension(required=True).uq8_seg_compress(x, x_off, q_off, lens, q, cb, int(x_end), int(q_end))
        return
    quant = Uniform8BitQuantization()
    for i, (xo, qo, n) in enumerate(zip(x_off.tolist(), q_off.tolist(), lens.tolist())):
        c = quant.compress(x[xo:xo + n])
        q[qo:qo + n] = c["idx"]
        cb[i * 256:(i + 1) * 256] = c["codebook"]


def _seg_dequant(q, q_off, cb, out_off, lens, out, q_end: int, out_end: int, accumulate=False):
    """``out[out_off[i]:+len[i]] (+)= cb[256 i + q[q_off[i]:+len[i]]]``."""
    if not lens.numel():
        return
    if q.is_cuda:
        from ..ops.ext import load_extension
        load_extension(required=True).uq8_seg_dequant_(q, q_off, cb, out_off, lens, out, 1.0, bool(accumulate),
                                                       int(q_end), int(out_end))
        return
    for i, (qo, oo, n) in enumerate(zip(q_off.tolist(), out_off.tolist(), lens.tolist())):
        v = cb[i * 256:(i + 1) * 256][q[qo:qo + n].long()]
        if accumulate:
            out[oo:oo + n] += v
        else:
            out[oo:oo + n] = v


def allreduce_weighted(x: torch.Tensor, weight: float, group=None, compression: Optional[CompressionBase] = None,
                       shard_weights: Optional[Sequence[float]] = None, total_weight: Optional[float] = None,
                       segments: Optional[Sequence[Tuple[int, int]]] = None) -> torch.Tensor:
    """Weighted average of the flat fp32 tensor ``x`` across ``group`` (in place).

    ``total_weight`` (sum of the weights) may be given when it is already known (e.g. from the
    progress tracker) to save one collective. ``segments`` = ``(offset, numel)`` of the tensors packed
    in ``x`` (compression is chosen and applied per tensor); default: ``x`` is one tensor."""
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
    return butterfly_allreduce(x, scale, group, compression, shard_weights, segments)


def butterfly_allreduce(x: torch.Tensor, scale: float, group, compression: CompressionBase,
                        shard_weights: Optional[Sequence[float]] = None,
                        segments: Optional[Sequence[Tuple[int, int]]] = None) -> torch.Tensor:
    """Compressed reduce-scatter + all-gather. ``x`` (flat fp32) is overwritten with the sum over peers
    of ``scale_p * x_p`` (scale_p = w_p / sum w)."""
    W, me = _world(group)
    flat = x.reshape(-1)
    assert flat.dtype == torch.float32 and flat.is_contiguous(), "butterfly: x must be a contiguous fp32 vector"
    n = flat.numel()
    plan = get_plan(n, segments if segments is not None else [(0, n)],
                    list(shard_weights) if shard_weights is not None else [1.0] * W, compression, flat.device)
    dev, edt = flat.device, plan.e_dtype
    contrib = flat * scale

    # ---------------- leg 1: each owner's parts, compressed, to that owner
    E_me, U_me, P_me = plan.e_sizes[me], plan.u_sizes[me], plan.p_counts[me]
    e_send = contrib.index_select(0, plan.e_idx_all)
    if edt == torch.float16:
        e_send = e_send.clamp_(-Float16Compression.FP16_MAX, Float16Compression.FP16_MAX)
    e_send = e_send.to(edt)
    e_recv = torch.empty(E_me * W, dtype=edt, device=dev)
    if sum(plan.e_sizes):
        dist.all_to_all_single(e_recv, e_send, [E_me] * W, plan.e_sizes, group=group)

    q_send = torch.empty(plan.u_total, dtype=torch.uint8, device=dev)
    cb_send = torch.empty(sum(plan.p_counts) * 256, dtype=torch.float32, device=dev)
    _seg_compress(contrib, plan.t_flat_off, plan.t_packed_off, plan.t_len, q_send, cb_send, plan.flat_end, plan.u_total)
    q_recv = torch.empty(U_me * W, dtype=torch.uint8, device=dev)
    cb_recv = torch.empty(P_me * 256 * W, dtype=torch.float32, device=dev)
    if plan.u_total:
        dist.all_to_all_single(q_recv, q_send, [U_me] * W, plan.u_sizes, group=group)
        dist.all_to_all_single(cb_recv, cb_send, [P_me * 256] * W, [p * 256 for p in plan.p_counts], group=group)

    # ---------------- reduce the own shard in fp32
    acc_e = e_recv.view(W, E_me).float().sum(0) if E_me else torch.zeros(0, dtype=torch.float32, device=dev)
    acc_u = torch.zeros(U_me, dtype=torch.float32, device=dev)
    rel, ln = plan.own_rel_off[me], plan.own_len[me]
    for src in range(W):
        _seg_dequant(q_recv[src * U_me:(src + 1) * U_me], rel, cb_recv[src * P_me * 256:(src + 1) * P_me * 256], rel, ln, acc_u,
                     U_me, U_me, accumulate=True)

    # ---------------- leg 2: averaged shard, compressed, to everyone (padded all-gather)
    E_max, U_max, P_max = max(plan.e_sizes), max(plan.u_sizes), max(plan.p_counts)
    mine_e = torch.zeros(E_max, dtype=edt, device=dev)
    if E_me:
        v = acc_e.clamp_(-Float16Compression.FP16_MAX, Float16Compression.FP16_MAX) if edt == torch.float16 else acc_e
        mine_e[:E_me] = v.to(edt)
    mine_q = torch.zeros(U_max, dtype=torch.uint8, device=dev)
    mine_cb = torch.zeros(P_max * 256, dtype=torch.float32, device=dev)
    _seg_compress(acc_u, rel, rel, ln, mine_q, mine_cb[:P_me * 256], U_me, U_me)
    all_e = torch.empty(E_max * W, dtype=edt, device=dev)
    all_q = torch.empty(U_max * W, dtype=torch.uint8, device=dev)
    all_cb = torch.empty(P_max * 256 * W, dtype=torch.float32, device=dev)
    if E_max:
        dist.all_gather_into_tensor(all_e, mine_e, group=group) if dev.type == "cuda" else \
            dist.all_gather(list(all_e.chunk(W)), mine_e, group=group)
    if U_max:
        if dev.type == "cuda":
            dist.all_gather_into_tensor(all_q, mine_q, group=group)
            dist.all_gather_into_tensor(all_cb, mine_cb, group=group)
        else:
            dist.all_gather(list(all_q.chunk(W)), mine_q, group=group)
            dist.all_gather(list(all_cb.chunk(W)), mine_cb, group=group)

    # ---------------- extract into place
    if E_max:
        vals = torch.cat([all_e[d * E_max:d * E_max + plan.e_sizes[d]] for d in range(W)]).float()
        flat.index_copy_(0, plan.e_idx_all, vals)
    for d in range(W):
        if plan.p_counts[d]:
            _seg_dequant(all_q[d * U_max:(d + 1) * U_max], plan.own_rel_off[d], all_cb[d * P_max * 256:d * P_max * 256 + plan.p_counts[d] * 256],
                         plan.own_flat_off[d], plan.own_len[d], flat, plan.u_sizes[d], plan.own_flat_end[d])
    return x


def broadcast_tensors(tensors: Sequence[torch.Tensor], src: int, group=None):
    """Broadcast a list of tensors from ``src`` (donor) -- used by load_state_from_peers (C3)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    for t in tensors:
        dist.broadcast(t, src=src, group=group)
