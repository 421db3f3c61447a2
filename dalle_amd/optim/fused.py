"""Fused multi-tensor LAMB over a :class:`FlatArena` (HIP path; kernels in ``csrc/optim/lamb.hip``).

State lives in arena-shaped buffers (uint8 moments for 8-bit tensors, fp32 moments for the small
ones, per-block absmax), and ``optimizer.state[p]`` holds *views* into them with the reference's key
names (``state1/state2/qmap1/qmap2/absmax1/absmax2/step/weight_norm/step_norm/trust_ratio``), so
``state_dict()`` / ``load_state_dict()`` keep the bnb-compatible per-parameter layout.
"""
from __future__ import annotations

import torch

from . import quant
from .flat import ALIGN


class FusedLambEngine:
    @staticmethod
    def maybe_create(opt):
        arena = getattr(opt, "arena", None)
        if arena is None or not arena.data.is_cuda:
            return None
        from ..ops.ext import load_extension
        load_extension(required=True)
        in_arena = {id(p) for p in arena.params}
        for g in opt.param_groups:
            for p in g["params"]:
                if id(p) not in in_arena:
                    return None
        if any(g["block_wise"] != ALIGN for g in opt.param_groups):
            return None
        betas = {tuple(g["betas"]) for g in opt.param_groups}
        eps = {g["eps"] for g in opt.param_groups}
        if len(betas) != 1 or len(eps) != 1:
            return None
        return FusedLambEngine(opt)

    def __init__(self, opt):
        from ..ops.ext import load_extension
        self.C = load_extension(required=True)
        self.opt = opt
        arena = self.arena = opt.arena
        dev = arena.data.device
        n, nb, nt = arena.numel, arena.numel // ALIGN, len(arena.params)
        self.q1 = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.q2 = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.absmax1 = torch.zeros(nb, dtype=torch.float32, device=dev)
        self.absmax2 = torch.zeros(nb, dtype=torch.float32, device=dev)
        self.m32 = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v32 = torch.zeros(n, dtype=torch.float32, device=dev)
        self.delta = torch.zeros(n, dtype=torch.float32, device=dev)
        self.partial = torch.zeros(2 * nb, dtype=torch.float32, device=dev)
        self.coef = torch.ones(1, dtype=torch.float32, device=dev)
        self.gnorm = torch.zeros(1, dtype=torch.float32, device=dev)
        self.trust = torch.ones(nt, dtype=torch.float32, device=dev)
        self.wnorm = torch.zeros(nt, dtype=torch.float32, device=dev)
        self.snorm = torch.zeros(nt, dtype=torch.float32, device=dev)
        self.code1 = quant.dynamic_map(True, dev)
        self.code2 = quant.dynamic_map(False, dev)
        self.tstart = arena.starts.to(dev)
        self.tsize = arena.sizes.to(dev)
        # per-tensor hyper-parameters from the param groups
        group_of = {}
        for gi, g in enumerate(opt.param_groups):
            for p in g["params"]:
                group_of[id(p)] = gi
        self.group_idx = [group_of[id(p)] for p in arena.params]
        modes = []
        for p in arena.params:
            g = opt.param_groups[group_of[id(p)]]
            modes.append(1 if opt._is_8bit(g, p) else 0)
        self.tmode = torch.tensor(modes, dtype=torch.int32, device=dev)
        self.twd = torch.tensor([opt.param_groups[gi]["weight_decay"] for gi in self.group_idx], dtype=torch.float32, device=dev)
        self.tlr = torch.zeros(nt, dtype=torch.float32, device=dev)
        self._lr_host = None
        self.step_count = 0
        self._bind_state()

    def _bind_state(self):
        opt, arena = self.opt, self.arena
        for i, (p, o) in enumerate(zip(arena.params, arena.offsets)):
            st = opt.state[p]
            k = p.numel()
            b0, b1 = o // ALIGN, (o + k + ALIGN - 1) // ALIGN
            st.setdefault("step", 0)
            if int(self.tmode[i]):
                st["state1"] = self.q1[o:o + k].view_as(p)
                st["state2"] = self.q2[o:o + k].view_as(p)
                st["qmap1"], st["qmap2"] = self.code1, self.code2
                st["absmax1"] = self.absmax1[b0:b1]
                st["absmax2"] = self.absmax2[b0:b1]
            else:
                st["state1"] = self.m32[o:o + k].view_as(p)
                st["state2"] = self.v32[o:o + k].view_as(p)
            st["weight_norm"] = self.wnorm[i]
            st["step_norm"] = self.snorm[i]
            st["trust_ratio"] = self.trust[i]

    def load_from_state(self):
        """After ``optimizer.load_state_dict``: copy loaded per-param tensors into the arenas."""
        opt, arena = self.opt, self.arena
        for i, (p, o) in enumerate(zip(arena.params, arena.offsets)):
            st = opt.state.get(p, {})
            k = p.numel()
            b0, b1 = o // ALIGN, (o + k + ALIGN - 1) // ALIGN
            if "state1" in st:
                if int(self.tmode[i]):
                    self.q1[o:o + k].copy_(st["state1"].reshape(-1))
                    self.q2[o:o + k].copy_(st["state2"].reshape(-1))
                    self.absmax1[b0:b1].copy_(st["absmax1"])
                    self.absmax2[b0:b1].copy_(st["absmax2"])
                else:
                    self.m32[o:o + k].copy_(st["state1"].reshape(-1).float())
                    self.v32[o:o + k].copy_(st["state2"].reshape(-1).float())
        self._bind_state()

    def _sync_lr(self):
        lrs = [float(self.opt.param_groups[gi]["lr"]) for gi in self.group_idx]
        if lrs != self._lr_host:
            self.tlr.copy_(torch.tensor(lrs, dtype=torch.float32), non_blocking=True)
            self._lr_host = lrs

    @torch.no_grad()
    def step(self):
        opt = self.opt
        g0 = opt.param_groups[0]
        beta1, beta2 = g0["betas"]
        self._sync_lr()
        use_clip = opt.max_grad_norm is not None
        if use_clip:
            self.C.lamb_grad_norm(self.arena.grad, self.partial, float(opt.max_grad_norm), self.coef, self.gnorm)
            opt.last_grad_norm = self.gnorm
        if opt.bias_correction:
            raise NotImplementedError("bias_correction=True is not supported by the fused path")
        self.C.lamb_step(self.arena.data, self.arena.grad, self.delta, self.q1, self.q2, self.absmax1, self.absmax2,
                         self.m32, self.v32, self.code1, self.code2, self.arena.block_tensor, self.tstart, self.tsize,
                         self.tmode, self.twd, self.tlr, self.coef, self.partial, self.trust, self.wnorm, self.snorm,
                         float(beta1), float(beta2), float(g0["eps"]), float(opt.clamp_value), use_clip)
        self.step_count += 1
        for p in self.arena.params:
            opt.state[p]["step"] = opt.state[p].get("step", 0) + 1
