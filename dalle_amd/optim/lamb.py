"""LAMB with blockwise 8-bit moments and baked-in global grad clipping.

API- and state-compatible with the reference's ``CPULAMB8Bit`` (``lib/training/lamb_8bit.py:13-250``):

* ctor ``(params, lr, betas, eps, weight_decay, clamp_value, bias_correction, min_8bit_size,
  reuse_grad_buffers, update_chunk_size, max_grad_norm)``; same argument validation (``:54-71``);
* ``step()`` clips all grads to ``max_grad_norm`` (``:83-88``), then per parameter:
  ``m = b1*m + (1-b1)*g``, ``v = b2*v + (1-b2)*g^2`` (dequantised from / requantised to uint8 with the
  signed / unsigned dynamic maps, 4096-element blocks), ``delta = m/(sqrt(v)+eps) + wd*p``,
  ``trust = clamp(|p|, 0, clamp_value) / |delta|`` (1 if either norm is 0), ``p -= lr*trust*delta``;
* tensors with fewer than ``min_8bit_size`` elements keep fp32 moments (``:106-111``);
* per-param state ``step, state1, state2, qmap1, qmap2, absmax1, absmax2, weight_norm, step_norm,
  trust_ratio``.

Execution: when the parameters live in a :class:`~dalle_amd.optim.flat.FlatArena` on a GPU the
whole step is three HIP launches over the arena (grad-norm reduction, fused
dequant->moments->requant->delta + per-tensor norm partials, trust-ratio apply) with no host sync
(``csrc/optim/lamb.hip``). Otherwise a per-tensor PyTorch path runs (CPU peers, tests) -- the
reference's "CPU offload" mode.
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..utils.logging import get_logger
from . import quant
from .flat import FlatArena

_logger = get_logger(__name__)


class LAMB8bit(torch.optim.Optimizer):
    def __init__(
        self,
        params,
        lr: float = 1e-3,
        betas=(0.9, 0.999),
        eps: float = 1e-6,
        weight_decay: float = 0.0,
        clamp_value: float = 10.0,
        bias_correction: bool = False,
        min_8bit_size: int = 65536,
        reuse_grad_buffers: bool = False,
        update_chunk_size: int = 2 ** 24,
        max_grad_norm: Optional[float] = None,
        optim_bits: int = 8,
        block_wise: int = quant.BLOCK,
        arena: Optional[FlatArena] = None,
    ):
        if lr <= 0.0:
            raise ValueError("Invalid learning rate: {}".format(lr))
        if eps < 0.0:
            raise ValueError("Invalid epsilon value: {}".format(eps))
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError("Invalid beta parameter at index 0: {}".format(betas[0]))
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError("Invalid beta parameter at index 1: {}".format(betas[1]))
        if weight_decay < 0:
            raise ValueError("Invalid weight_decay value: {}".format(weight_decay))
        if clamp_value < 0.0:
            raise ValueError("Invalid clamp value: {}".format(clamp_value))
        if optim_bits not in (8, 32):
            raise NotImplementedError(f"Amount of optimizer bits not supported: {optim_bits}")
        # non-group options (CPULAMB8Bit keeps them as attributes; state_dict compatibility needs the names)
        for name, val in (("clamp_value", clamp_value), ("bias_correction", bias_correction),
                          ("reuse_grad_buffers", reuse_grad_buffers), ("update_chunk_size", update_chunk_size),
                          ("max_grad_norm", max_grad_norm)):
            setattr(self, name, val)
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, optim_bits=optim_bits,
                        min_8bit_size=min_8bit_size, percentile_clipping=100, block_wise=block_wise, max_unorm=0.0)
        super().__init__(params, defaults)
        self.arena = arena
        self._fused = None
        self.name2qmap = {}
        self.last_grad_norm = None

    # ------------------------------------------------------------------------------------------
    def fill_qmap(self):
        self.name2qmap["dynamic"] = quant.dynamic_map(True)
        self.name2qmap["udynamic"] = quant.dynamic_map(False)

    def _is_8bit(self, group, p) -> bool:
        return group["optim_bits"] == 8 and p.numel() >= group["min_8bit_size"] and p.numel() >= 4096

    @torch.no_grad()
    def init_state(self, group, p):
        state = self.state[p]
        state["step"] = 0
        if not self._is_8bit(group, p):
            state["state1"] = torch.zeros_like(p, dtype=torch.float32)
            state["state2"] = torch.zeros_like(p, dtype=torch.float32)
        else:
            if "dynamic" not in self.name2qmap:
                self.fill_qmap()
            self.name2qmap["dynamic"] = self.name2qmap["dynamic"].to(p.device)
            self.name2qmap["udynamic"] = self.name2qmap["udynamic"].to(p.device)
            nb = quant.num_blocks(p.numel(), group["block_wise"])
            state["state1"] = torch.zeros_like(p, dtype=torch.uint8)
            state["qmap1"] = self.name2qmap["dynamic"]
            state["state2"] = torch.zeros_like(p, dtype=torch.uint8)
            state["qmap2"] = self.name2qmap["udynamic"]
            state["absmax1"] = torch.zeros((nb,), dtype=torch.float32, device=p.device)
            state["absmax2"] = torch.zeros((nb,), dtype=torch.float32, device=p.device)

    def load_state_dict(self, state_dict):
        """torch casts every floating param's state to the param dtype; keep the uint8 moments uint8."""
        super().load_state_dict(state_dict)
        for st in self.state.values():
            if "qmap1" in st:
                st["state1"] = st["state1"].to(torch.uint8)
                st["state2"] = st["state2"].to(torch.uint8)
        if self._fused:
            self._fused.load_from_state()

    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def clip_grad_norm_(self):
        params = [p for g in self.param_groups for p in g["params"] if p.grad is not None]
        if self.max_grad_norm is None or not params:
            return None
        norm = torch.nn.utils.clip_grad_norm_(params, self.max_grad_norm)
        self.last_grad_norm = norm
        return norm

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        fused = self._get_fused()
        if fused is not None:
            fused.step()
            return loss
        self.clip_grad_norm_()
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p not in self.state or "step" not in self.state[p]:
                    self.init_state(group, p)
                self.update_step(group, p)
        return loss

    def _get_fused(self):
        if self._fused is False:
            return None
        if self._fused is None:
            from .fused import FusedLambEngine
            self._fused = FusedLambEngine.maybe_create(self) or False
            if self._fused is False:
                if any(p.is_cuda for g in self.param_groups for p in g["params"]):
                    _logger.info("LAMB: per-tensor PyTorch path (parameters outside a flat arena)")
                return None
            _logger.info(f"LAMB: fused HIP engine over the flat arena ({self.defaults['optim_bits']}-bit state, "
                         f"{self._fused.state_bytes() / 2 ** 20:.1f} MiB)")
        return self._fused

    @torch.no_grad()
    def update_step(self, group, p):
        state = self.state[p]
        state["step"] += 1
        step = state["step"]
        beta1, beta2 = group["betas"]
        delta = self._moments_and_delta(state, group, p, p.grad, beta1, beta2, group["eps"], group["weight_decay"])
        step_norm = torch.norm(delta)
        weight_norm = p.norm().clamp(0, self.clamp_value)
        trust_ratio = weight_norm / step_norm if weight_norm != 0 and step_norm != 0 else torch.ones((), device=p.device)
        state["weight_norm"], state["step_norm"], state["trust_ratio"] = weight_norm, step_norm, trust_ratio
        bc = math.sqrt(1 - beta2 ** step) / (1 - beta1 ** step) if self.bias_correction else 1.0
        p.add_(delta.to(p.dtype) * (-group["lr"] * bc * trust_ratio))

    def _moments_and_delta(self, state, group, p, grad, beta1, beta2, eps, weight_decay):
        grad = grad.float()
        if state["state1"].dtype != torch.uint8:
            m, v = state["state1"], state["state2"]
            m.mul_(beta1).add_(grad, alpha=1 - beta1)
            v.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
            delta = m / (v.sqrt() + eps)
        else:
            bw = group["block_wise"]
            m = quant.dequantize_blockwise(state["state1"], state["absmax1"], state["qmap1"], bw)
            v = quant.dequantize_blockwise(state["state2"], state["absmax2"], state["qmap2"], bw)
            m.mul_(beta1).add_(grad, alpha=1 - beta1)
            v.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
            q1, a1 = quant.quantize_blockwise(m, state["qmap1"], bw)
            q2, a2 = quant.quantize_blockwise(v, state["qmap2"], bw)
            state["state1"].copy_(q1)
            state["state2"].copy_(q2)
            state["absmax1"].copy_(a1)
            state["absmax2"].copy_(a2)
            delta = m.div_(v.sqrt_().add_(eps))
        if weight_decay != 0:
            delta = delta + weight_decay * p.float()
        return delta


# The reference names (`lib/training/lamb_8bit.py:13`, `lib/training/clipped_lamb.py:5`)
CPULAMB8Bit = LAMB8bit


def LambWithGradientClipping(params, max_grad_norm: float, **kwargs):
    """fp32-moment LAMB + global clip (``lib/training/clipped_lamb.py:5-14``)."""
    kwargs.setdefault("clamp_value", 10.0)
    return LAMB8bit(params, max_grad_norm=max_grad_norm, optim_bits=32, **kwargs)
