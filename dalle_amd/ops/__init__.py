"""Op dispatch: hand-written HIP/CDNA4 kernels on MI355X, pure-PyTorch reference on CPU.

Every op the model calls goes through this module. Backend selection per call:

* CPU tensors                    -> ``reference`` (pure PyTorch, fp32)
* CUDA(=HIP) tensors              -> ``hip`` (``dalle_amd._C`` kernels + hipBLASLt GEMMs), bf16 compute
* ``DALLE_AMD_BACKEND=torch``     -> force the reference ops on GPU too (A/B and numerics checks)

On a GPU the HIP extension is REQUIRED: if ``dalle_amd._C`` cannot be imported the first GPU op
raises instead of silently running the eager fallback.
"""
from __future__ import annotations

import os

import torch

from . import reference
from .ext import hip_available, load_extension  # noqa: F401

COMPUTE_DTYPE = torch.bfloat16


def backend_for(t: torch.Tensor) -> str:
    forced = os.environ.get("DALLE_AMD_BACKEND", "auto")
    if not t.is_cuda:
        return "torch"
    if forced == "torch":
        return "torch_gpu"
    load_extension(required=True)
    return "hip"


def _hip():
    from . import hip_ops
    return hip_ops


# ---------------------------------------------------------------------------------------------
def layernorm_shift(x, weight, bias, text_len: int, image_size: int, shift: bool = True):
    be = backend_for(x)
    if be == "torch":
        return reference.layernorm_shift(x, weight, bias, text_len, image_size, shift)
    if be == "torch_gpu":
        return reference.layernorm_shift(x, weight, bias, text_len, image_size, shift).to(COMPUTE_DTYPE)
    return _hip().layernorm_shift(x, weight, bias, text_len, image_size, shift)


def attention_block(h, w_qkv, w_out, b_out, heads: int, geom, attn_type: str):
    be = backend_for(h)
    if be == "hip":
        return _hip().attention_block(h, w_qkv, w_out, b_out, heads, geom, attn_type)
    from ..models.rotary import rotary_tables
    cos, sin = rotary_tables(geom.text_len, geom.image_size, w_qkv.shape[0] // 3 // heads, device=h.device)
    if be == "torch_gpu":
        dt = COMPUTE_DTYPE
        return reference.attention_block(h.to(dt), w_qkv.to(dt), w_out.to(dt), b_out.to(dt), heads, geom, attn_type, cos, sin)
    return reference.attention_block(h, w_qkv, w_out, b_out, heads, geom, attn_type, cos, sin)


def feed_forward(h, w1, b1, w2, b2):
    be = backend_for(h)
    if be == "hip":
        return _hip().feed_forward(h, w1, b1, w2, b2)
    if be == "torch_gpu":
        dt = COMPUTE_DTYPE
        return reference.feed_forward(h.to(dt), w1.to(dt), b1.to(dt), w2.to(dt), b2.to(dt))
    return reference.feed_forward(h, w1, b1, w2, b2)


def attention_out(h, w_qkv, heads: int, geom, attn_type: str):
    """QKV projection + rotary + sparse attention, before the output projection."""
    be = backend_for(h)
    if be == "hip":
        return _hip().attention_out(h, w_qkv, heads, geom, attn_type)
    from ..models.rotary import rotary_tables
    cos, sin = rotary_tables(geom.text_len, geom.image_size, w_qkv.shape[0] // 3 // heads, device=h.device)
    dt = COMPUTE_DTYPE if be == "torch_gpu" else h.dtype
    qkv = torch.nn.functional.linear(h.to(dt), w_qkv.to(dt))
    q, k, v = reference.qkv_rotary(qkv, heads, cos, sin)
    return reference.sparse_attention_core(q, k, v, geom, attn_type)


def ff_hidden(h, w1, b1):
    """FF-in projection + GEGLU (the FF block before its output projection)."""
    be = backend_for(h)
    if be == "hip":
        return _hip().ff_hidden(h, w1, b1)
    dt = COMPUTE_DTYPE if be == "torch_gpu" else h.dtype
    return reference.geglu(torch.nn.functional.linear(h.to(dt), w1.to(dt), b1.to(dt)))


def proj_residual(x, o, w, b, scale):
    """x + scale * (o W^T + b): output projection with the LayerScale residual epilogue."""
    be = backend_for(x)
    if be == "hip":
        return _hip().proj_residual(x, o, w, b, scale)
    dt = o.dtype
    y = torch.nn.functional.linear(o, w.to(dt), b.to(dt))
    return x + (y * scale.to(dt)).to(x.dtype)


def attn_sublayer(x, ln_w, ln_b, w_qkv, w_out, b_out, scale, heads: int, geom, attn_type: str, shift: bool):
    """x + LayerScale * Attention(PreShiftToken(LayerNorm(x))) -- one fused autograd node on HIP."""
    if backend_for(x) == "hip":
        return _hip().attn_sublayer(x, ln_w, ln_b, w_qkv, w_out, b_out, scale, heads, geom, attn_type, shift)
    h = layernorm_shift(x, ln_w, ln_b, geom.text_len, geom.image_size, shift)
    return proj_residual(x, attention_out(h, w_qkv, heads, geom, attn_type), w_out, b_out, scale)


def ff_sublayer(x, ln_w, ln_b, w1, b1, w2, b2, scale, text_len: int, image_size: int, shift: bool):
    """x + LayerScale * FeedForward(PreShiftToken(LayerNorm(x))) -- one fused autograd node on HIP."""
    if backend_for(x) == "hip":
        return _hip().ff_sublayer(x, ln_w, ln_b, w1, b1, w2, b2, scale, text_len, image_size, shift)
    h = layernorm_shift(x, ln_w, ln_b, text_len, image_size, shift)
    return proj_residual(x, ff_hidden(h, w1, b1), w2, b2, scale)


def attn_meta(x, w_qkv, heads: int, geom, attn_type: str, shift: bool):
    """Per-sublayer constants of the fused attention core: (heads, cos, sin, meta)."""
    return _hip().attn_args(x, w_qkv, heads, geom, attn_type, shift)


def sequential_stack(x, subs):
    """Non-reversible layer stack as one fused HIP autograd node (``hip_ops.sequential_stack``), or None
    when it does not apply (CPU, no flat-arena grad buffers): the caller runs the sublayers one by one."""
    if not (x.is_cuda and backend_for(x) == "hip" and torch.is_grad_enabled()):
        return None
    return _hip().sequential_stack(x, subs)


FUSED_REVERSIBLE = True  # False: the reversible stack over per-op autograd nodes (numerics A/B in tests)


def fused_reversible_available(x) -> bool:
    """True when the reversible stack can run on the fused HIP sublayers (``hip_ops.reversible_stack``)."""
    return x.is_cuda and backend_for(x) == "hip" and FUSED_REVERSIBLE


def reversible_stack(x, layers, geom, text_len: int, image_size: int, recompute: bool = True):
    """Reversible residual stack over the fused attention / FF sublayers (HIP only)."""
    return _hip().reversible_stack(x, layers, geom, text_len, image_size, recompute)


def begin_forward():
    """Start of a model forward: drops the per-forward bf16 weight casts of the HIP path."""
    if hip_available():
        _hip().begin_forward()


def scale_rows(o, scale):
    """LayerScale multiply (reversible branches; fused into the residual add otherwise)."""
    return o * scale.to(o.dtype)


def scale_residual(x, o, scale):
    """x + scale * o  -- residual add with the LayerScale fused in (K8/K10 epilogue)."""
    if x.is_cuda and backend_for(x) == "hip":
        return _hip().scale_residual(x, o, scale)
    return x + (o * scale.to(o.dtype)).to(x.dtype)


def grads_finite(buf: torch.Tensor) -> bool:
    """K17: one fused NaN/Inf check over a flat fp32 buffer (HIP kernel on GPU)."""
    if buf.is_cuda and backend_for(buf) == "hip":
        return int(_hip().nonfinite_flag(buf).item()) == 0
    return bool(torch.isfinite(buf).all())


def embed_tokens(text, image, weight, pad_base: int, Vt: int):
    """K1 + K2 on the HIP path (tied table); None on other backends (the caller gathers with F.embedding)."""
    if text.is_cuda and backend_for(text) == "hip" and weight.dtype == torch.float32:
        return _hip().embed_tokens(text, image, weight, pad_base, Vt)
    return None


def zero_grads_if_nonfinite_(buf: torch.Tensor) -> torch.Tensor:
    """Zero a flat fp32 gradient buffer iff it holds a NaN/Inf, entirely on the device (no host sync):
    the trainer's guarded ``zero_grad`` (``lib/training/hf_trainer.py:73-78``). Returns the flag tensor."""
    if buf.is_cuda and backend_for(buf) == "hip":
        return _hip().zero_if_nonfinite_(buf)
    bad = ~torch.isfinite(buf).all()
    buf.mul_((~bad).to(buf.dtype)).nan_to_num_(0.0, 0.0, 0.0)
    return bad.to(torch.int32).reshape(1)


def residual_add(x, y):
    return x + y.to(x.dtype)


def logits_loss(out, norm_w, norm_b, weight, bias, labels, text_seq_len: int, num_text_tokens: int, loss_img_weight: float):
    be = backend_for(out)
    if be == "hip":
        return _hip().logits_loss(out, norm_w, norm_b, weight, bias, labels, text_seq_len, num_text_tokens, loss_img_weight)
    h = torch.nn.functional.layer_norm(out, (out.shape[-1],), norm_w, norm_b)
    if be == "torch_gpu":
        dt = COMPUTE_DTYPE
        return reference.split_logits_loss(h.to(dt), weight.to(dt), bias.to(dt), labels, text_seq_len, num_text_tokens, loss_img_weight)
    return reference.split_logits_loss(h, weight, bias, labels, text_seq_len, num_text_tokens, loss_img_weight)
