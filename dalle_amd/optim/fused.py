"""Fused multi-tensor LAMB over a :class:`FlatArena` (HIP path; kernels in ``csrc/optim/lamb.hip``).

State lives in compact per-mode buffers (uint8 moments + per-block absmax for the 8-bit tensors,
fp32 moments only for the small fp32-state tensors: ~2 B/param + 8 B per 4096-block, the
reference's footprint; no fp32 delta buffer -- the apply pass recomputes it), and ``optimizer.state[p]`` holds *views* into them with the reference's key
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
        group_of = {}
        for gi, g in enumerate(opt.param_groups):
            for p in g["params"]:
                group_of[id(p)] = gi
        self.group_idx = [group_of[id(p)] for p in arena.params]
        modes = [1 if opt._is_8bit(opt.param_groups[group_of[id(p)]], p) else 0 for p in arena.params]
        # compact per-mode state: a tensor's blocks take consecutive slots of its mode's arrays, so the
        # per-parameter views below stay contiguous (bnb layout) and no byte is spent on the other mode
        slots = torch.empty(nb, dtype=torch.int32)
        self.slot0 = []
        count = [0, 0]  # fp32 blocks, 8-bit blocks
        for i, (p, o) in enumerate(zip(arena.params, arena.offsets)):
            k = (p.numel() + ALIGN - 1) // ALIGN
            s0 = count[modes[i]]
            self.slot0.append(s0)
            slots[o // ALIGN:o // ALIGN + k] = torch.arange(s0, s0 + k, dtype=torch.int32)
            count[modes[i]] += k
        self.n32_blocks, self.n8_blocks = count
        assert self.n32_blocks + self.n8_blocks == nb
        self.bslot = slots.to(dev)
        self.q1 = torch.zeros(self.n8_blocks * ALIGN, dtype=torch.uint8, device=dev)
        self.q2 = torch.zeros(self.n8_blocks * ALIGN, dtype=torch.uint8, device=dev)
        self.absmax1 = torch.zeros(self.n8_blocks, dtype=torch.float32, device=dev)
        self.absmax2 = torch.zeros(self.n8_blocks, dtype=torch.float32, device=dev)
        self.m32 = torch.zeros(self.n32_blocks * ALIGN, dtype=torch.float32, device=dev)
        self.v32 = torch.zeros(self.n32_blocks * ALIGN, dtype=torch.float32, device=dev)
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
        self.tmode = torch.tensor(modes, dtype=torch.int32, device=dev)
        self.modes = modes
        self.twd = torch.tensor([opt.param_groups[gi]["weight_decay"] for gi in self.group_idx], dtype=torch.float32, device=dev)
        self.tlr = torch.zeros(nt, dtype=torch.float32, device=dev)
        self._lr_host = None
        self.step_count = 0
        # state restored (load_state_dict / load_state_from_peers) before the engine existed lands in
        # the arenas instead of being replaced by zeros
        if any("state1" in opt.state.get(p, {}) for p in arena.params):
            self.load_from_state()
        else:
            self._bind_state()

    def state_bytes(self) -> int:
        """HBM held by the optimizer state (moments + absmax), excluding the small per-tensor scalars."""
        return sum(t.numel() * t.element_size() for t in (self.q1, self.q2, self.absmax1, self.absmax2, self.m32, self.v32))

    def _views(self, i, p):
        k = p.numel()
        s0 = self.slot0[i]
        nblk = (k + ALIGN - 1) // ALIGN
        if self.modes[i]:
            return (self.q1[s0 * ALIGN:s0 * ALIGN + k].view_as(p), self.q2[s0 * ALIGN:s0 * ALIGN + k].view_as(p),
                    self.absmax1[s0:s0 + nblk], self.absmax2[s0:s0 + nblk])
        return self.m32[s0 * ALIGN:s0 * ALIGN + k].view_as(p), self.v32[s0 * ALIGN:s0 * ALIGN + k].view_as(p), None, None

    def _bind_state(self):
        opt, arena = self.opt, self.arena
        for i, p in enumerate(arena.params):
            st = opt.state[p]
            st.setdefault("step", 0)
            s1, s2, a1, a2 = self._views(i, p)
            st["state1"], st["state2"] = s1, s2
            if self.modes[i]:
                st["qmap1"], st["qmap2"] = self.code1, self.code2
                st["absmax1"], st["absmax2"] = a1, a2
            st["weight_norm"] = self.wnorm[i]
            st["step_norm"] = self.snorm[i]
            st["trust_ratio"] = self.trust[i]

    def load_from_state(self):
        """After ``optimizer.load_state_dict`` (or before the first step): copy the per-param tensors
        found in ``optimizer.state`` into the arenas, then bind the views."""
        opt, arena = self.opt, self.arena
        for i, p in enumerate(arena.params):
            st = opt.state.get(p, {})
            if "state1" not in st:
                continue
            s1, s2, a1, a2 = self._views(i, p)
            if self.modes[i]:
                s1.copy_(st["state1"].reshape(s1.shape).to(torch.uint8))
                s2.copy_(st["state2"].reshape(s2.shape).to(torch.uint8))
                a1.copy_(st["absmax1"].reshape(-1))
                a2.copy_(st["absmax2"].reshape(-1))
            else:
                s1.copy_(st["state1"].reshape(s1.shape).float())
                s2.copy_(st["state2"].reshape(s2.shape).float())
            for key, buf in (("weight_norm", self.wnorm), ("step_norm", self.snorm), ("trust_ratio", self.trust)):
                if key in st and torch.is_tensor(st[key]):
                    buf[i].copy_(st[key].reshape(()))
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
        self.C.lamb_step(self.arena.data, self.arena.grad, self.q1, self.q2, self.absmax1, self.absmax2,
                         self.m32, self.v32, self.code1, self.code2, self.arena.block_tensor, self.bslot, self.tstart,
                         self.tsize, self.tmode, self.twd, self.tlr, self.coef, self.partial, self.trust, self.wnorm,
                         self.snorm, self.n8_blocks, self.n32_blocks, float(beta1), float(beta2), float(g0["eps"]),
                         float(opt.clamp_value), use_clip)
        self.step_count += 1
        for p in self.arena.params:
            opt.state[p]["step"] = opt.state[p].get("step", 0) + 1
