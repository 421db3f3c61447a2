"""Pure-PyTorch reference implementations of every fused op.

These encode the semantics the HIP kernels must reproduce and serve as (a) the CPU execution
path used by the plumbing tests / CPU peers and (b) the fp32 golden for kernel numerics tests.
Every op here is autograd-differentiable through plain torch ops.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..models.patterns import AttnGeometry, static_mask
from ..models.rotary import apply_rotary


# --------------------------------------------------------------------------------------------
# K3 + K4: LayerNorm followed by token shift (PreNorm -> PreShiftToken)
# --------------------------------------------------------------------------------------------
def token_shift(x: torch.Tensor, text_len: int, image_size: int) -> torch.Tensor:
    """x (B, n, D). Text: first half of channels from the previous position. Image (raster order):
    first quarter from the token above, second quarter from the token to the left, rest pass."""
    B, n, D = x.shape
    if n < text_len:
        return x
    S = image_size
    x_text, x_img = x[:, :text_len], x[:, text_len:]
    half = D // 2
    t_shift = F.pad(x_text[..., :half], (0, 0, 1, -1))
    x_text = torch.cat([t_shift, x_text[..., half:]], dim=-1)

    n_img = x_img.shape[1]
    pad = S * S - n_img
    x_img = F.pad(x_img, (0, 0, 0, pad)).reshape(B, S, S, D)
    q = D // 4
    top = F.pad(x_img[..., :q], (0, 0, 0, 0, 1, -1))
    left = F.pad(x_img[..., q:2 * q], (0, 0, 1, -1))
    x_img = torch.cat([top, left, x_img[..., 2 * q:]], dim=-1).reshape(B, S * S, D)[:, :n_img]
    return torch.cat([x_text, x_img], dim=1)


def layernorm_shift(x, weight, bias, text_len: int, image_size: int, shift: bool = True, eps: float = 1e-5):
    y = F.layer_norm(x, (x.shape[-1],), weight, bias, eps)
    if shift:
        y = token_shift(y, text_len, image_size)
    return y


# --------------------------------------------------------------------------------------------
# K5-K8: attention block (QKV projection, 3-axis rotary on q/k/v, sparse attention, out proj)
# --------------------------------------------------------------------------------------------
def split_heads(t: torch.Tensor, heads: int) -> torch.Tensor:
    B, n, HD = t.shape
    return t.view(B, n, heads, HD // heads).transpose(1, 2)


def qkv_rotary(qkv: torch.Tensor, heads: int, cos: torch.Tensor, sin: torch.Tensor):
    """qkv (B, n, 3*H*D) -> rotated q (pre-scaled by D**-0.5), k, v, each (B, H, n, D)."""
    n = qkv.shape[1]
    q, k, v = qkv.chunk(3, dim=-1)
    q, k, v = (split_heads(t, heads) for t in (q, k, v))
    c, s = cos[:n].to(qkv.dtype), sin[:n].to(qkv.dtype)
    q, k, v = (apply_rotary(t, c, s) for t in (q, k, v))
    q = q * (q.shape[-1] ** -0.5)
    return q, k, v


def sparse_attention_core(q, k, v, geom: AttnGeometry, attn_type: str):
    """q (pre-scaled), k, v: (B, H, n, D) -> (B, n, H*D); dense masked softmax in fp32."""
    B, H, n, D = q.shape
    mask = static_mask(geom, attn_type, n, device=q.device)
    scores = torch.matmul(q.float(), k.float().transpose(-1, -2))
    scores = scores.masked_fill(~mask, -torch.finfo(torch.float32).max)
    p = torch.softmax(scores, dim=-1)
    out = torch.matmul(p, v.float()).to(q.dtype)
    return out.transpose(1, 2).reshape(B, n, H * D)


def attention_block(x_normed, w_qkv, w_out, b_out, heads: int, geom: AttnGeometry, attn_type: str, cos, sin):
    qkv = F.linear(x_normed, w_qkv)
    q, k, v = qkv_rotary(qkv, heads, cos, sin)
    o = sparse_attention_core(q, k, v, geom, attn_type)
    return F.linear(o, w_out, b_out)


# --------------------------------------------------------------------------------------------
# K9-K10: GEGLU feed-forward
# --------------------------------------------------------------------------------------------
def geglu(h: torch.Tensor) -> torch.Tensor:
    a, g = h.chunk(2, dim=-1)
    return a * F.gelu(g)


def feed_forward(x_normed, w1, b1, w2, b2):
    return F.linear(geglu(F.linear(x_normed, w1, b1)), w2, b2)


# --------------------------------------------------------------------------------------------
# K12: final LayerNorm + split (masked) logits + cross entropy (D1)
# --------------------------------------------------------------------------------------------
def split_logits_loss(h, weight, bias, labels, text_seq_len: int, num_text_tokens: int, loss_img_weight: float):
    """h: (B, n, d) final-normed hidden; weight/bias of the tied (V, d) head; labels (B, n) in the
    global vocabulary. Text rows only see the text vocabulary, image rows the image vocabulary,
    which is exactly the reference's ``logits.masked_fill_(logits_mask, -max)``."""
    Vt = num_text_tokens
    h_t, h_i = h[:, :text_seq_len], h[:, text_seq_len:]
    lt = F.linear(h_t, weight[:Vt], bias[:Vt]).float()
    li = F.linear(h_i, weight[Vt:], bias[Vt:]).float()
    loss_t = F.cross_entropy(lt.reshape(-1, lt.shape[-1]), labels[:, :text_seq_len].reshape(-1))
    loss_i = F.cross_entropy(li.reshape(-1, li.shape[-1]), (labels[:, text_seq_len:] - Vt).reshape(-1))
    return (loss_t + loss_img_weight * loss_i) / (loss_img_weight + 1)


def masked_logits(h, weight, bias, text_seq_len: int, num_text_tokens: int, offset: int = 0):
    """Full logits with the static text/image mask applied (generation path)."""
    logits = F.linear(h, weight, bias).float()
    n = h.shape[1]
    pos = torch.arange(offset, offset + n, device=h.device).view(1, n, 1)
    vocab = torch.arange(weight.shape[0], device=h.device).view(1, 1, -1)
    mask = ((pos >= text_seq_len) & (vocab < num_text_tokens)) | ((pos < text_seq_len) & (vocab >= num_text_tokens))
    return logits.masked_fill(mask, -torch.finfo(torch.float32).max)
