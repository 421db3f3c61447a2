"""PowerSGD low-rank gradient compression with error feedback (BASELINE config 3).

Per 2-D gradient M (n x m) with error buffer E and a persistent right factor Q (m x r):

    M_e = M + E
    P   = M_e Q          -> all-reduce (mean)  -> orthonormalise columns (QR)
    Q   = M_e^T P        -> all-reduce (mean)
    M^  = P Q^T          (the averaged low-rank gradient);   E = M_e - M^

All P factors of a step travel in ONE all-reduce and all Q factors in a second one (two small RCCL
collectives per averaging round instead of 126M fp32 elements); 1-D / small tensors are averaged
uncompressed in a third flat all-reduce. The skinny GEMMs run on hipBLASLt. Sample weighting is
folded into a per-peer pre-scale so the mean is the weighted mean.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist


class PowerSGD:
    def __init__(self, params: List[torch.nn.Parameter], rank: int = 4, min_compression_ratio: float = 2.0,
                 seed: int = 0, group=None, error_feedback: bool = True):
        self.rank = rank
        self.group = group
        self.error_feedback = error_feedback
        self.low_rank, self.plain = [], []
        for p in params:
            if p.dim() >= 2:
                n, m = p.shape[0], p.numel() // p.shape[0]
                if (n * m) / ((n + m) * rank) >= min_compression_ratio:
                    self.low_rank.append(p)
                    continue
            self.plain.append(p)
        g = torch.Generator().manual_seed(seed)  # identical Q init on every peer
        self.Q = []
        self.E = []
        for p in self.low_rank:
            m = p.numel() // p.shape[0]
            self.Q.append(torch.randn(m, rank, generator=g).to(p.device))
            self.E.append(torch.zeros(p.shape[0], m, dtype=torch.float32, device=p.device) if error_feedback else None)

    def compression_ratio(self) -> float:
        full = sum(p.numel() for p in self.low_rank) + sum(p.numel() for p in self.plain)
        sent = sum((p.shape[0] + p.numel() // p.shape[0]) * self.rank for p in self.low_rank) + sum(p.numel() for p in self.plain)
        return full / max(sent, 1)

    def _allreduce_mean(self, flat: torch.Tensor, world: int):
        if world > 1:
            dist.all_reduce(flat, group=self.group)
            flat.div_(world)

    def _native(self) -> bool:
        """HIP path: fused Gram-Schmidt + reconstruction kernels (csrc/kernels/powersgd.hip)."""
        if not self.low_rank or not self.low_rank[0].is_cuda or self.rank not in (1, 2, 4, 8):
            return False
        from ..ops.ext import load_extension
        self._C = load_extension(required=True)
        return all(p.grad is not None and p.grad.dtype == torch.float32 and p.grad.is_contiguous()
                   and (p.numel() // p.shape[0]) % 4 == 0 for p in self.low_rank)

    @torch.no_grad()
    def allreduce_(self, grads: Optional[List[torch.Tensor]] = None, scale: float = 1.0):
        """Average the ``.grad`` of the managed params in place (weighted by ``scale`` per peer:
        pass ``w_p * world / sum(w)`` for a sample-weighted mean)."""
        world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        native = self._native()
        r = self.rank
        # M_e = scale * grad (+ E): accumulated in place into the error buffer
        Ms = []
        for i, p in enumerate(self.low_rank):
            g = p.grad.reshape(p.shape[0], -1)
            if self.error_feedback:
                Ms.append(self.E[i].add_(g.float(), alpha=scale))
            else:
                Ms.append(g.float() * scale)
        if Ms:
            dev = Ms[0].device
            rows = [M.shape[0] for M in Ms]
            cols = [M.shape[1] for M in Ms]
            flatP = torch.empty(sum(rows) * r, dtype=torch.float32, device=dev)
            Ps, off = [], 0
            for M, Q, n in zip(Ms, self.Q, rows):
                P = flatP[off:off + n * r].view(n, r)
                torch.mm(M, Q, out=P)  # P = M Q
                Ps.append(P)
                off += n * r
            self._allreduce_mean(flatP, world)
            if native:
                offs = torch.tensor([0] + [n * r for n in rows[:-1]], dtype=torch.int64).cumsum(0).to(dev)
                self._C.psgd_orthonormalize_(flatP, offs, torch.tensor(rows, dtype=torch.int32, device=dev), r, 1e-8)
            else:
                for P in Ps:
                    P.copy_(torch.linalg.qr(P, mode="reduced")[0])
            flatQ = torch.empty(sum(cols) * r, dtype=torch.float32, device=dev)
            Qs, off = [], 0
            for M, P, m in zip(Ms, Ps, cols):
                Qn = flatQ[off:off + m * r].view(m, r)
                torch.mm(M.t(), P, out=Qn)  # Q = M^T P
                Qs.append(Qn)
                off += m * r
            self._allreduce_mean(flatQ, world)
            self.Q = Qs
            # reconstruct M^ = P Q^T into .grad; error feedback E = M_e - M^
            for p, M, P, Qn in zip(self.low_rank, Ms, Ps, Qs):
                if native:
                    self._C.psgd_reconstruct_(p.grad, M, P, Qn)
                else:
                    approx = P @ Qn.t()
                    if self.error_feedback:
                        M.sub_(approx)
                    p.grad.copy_(approx.view_as(p.grad))
        # --- small / 1-D tensors uncompressed
        if self.plain:
            flat = torch.cat([p.grad.reshape(-1).float() * scale for p in self.plain])
            self._allreduce_mean(flat, world)
            off = 0
            for p in self.plain:
                k = p.numel()
                p.grad.copy_(flat[off:off + k].view_as(p.grad))
                off += k

    def state_dict(self):
        return {"Q": [q.cpu() for q in self.Q], "E": [e.cpu() if e is not None else None for e in self.E]}

    def load_state_dict(self, sd):
        self.Q = [q.to(p.device) for q, p in zip(sd["Q"], self.low_rank)]
        self.E = [e.to(p.device) if e is not None else None for e, p in zip(sd["E"], self.low_rank)]
