"""3-axis rotary position embedding tables (``rotary_emb=True`` at ``task.py:80``).

Layout (dalle-pytorch Transformer with rotary-embedding-torch, [ext]):
  rot_dim = dim_head // 3 (= 21)
  * text 1-D frequencies: ``1 / 10000 ** (arange(0, rot_dim, 2) / rot_dim)`` -> 11 freqs -> 22 dims;
    text positions 0..text_len-1, image tokens get text position 8192.
  * image 2-D axial "pixel" frequencies: ``logspace(0, log2(max_freq/2), rot_dim // 2, base=2) * pi``
    (max_freq = 10) -> 10 freqs per axis -> 2 x 20 dims, positions ``linspace(-1, 1, image_size)``;
    text tokens get axial position -10 on both axes.
  * Concatenated = 62 of 64 head dims rotated, interleaved pairs ``(2i, 2i+1)`` share a frequency
    (``rotate_half`` on ``(d r) r=2``). The exact frequency family of the pinned fork could not be
    fetched offline: parity of the frequency values is *unpinned*, the layout (22 + 40 dims,
    interleaved, applied to q, k **and** v) follows SURVEY D4/D7.

Tables are returned as ``cos, sin`` of shape ``(n + 1, dim_head)`` fp32 (the padding token incl.),
with ``cos = 1, sin = 0`` on un-rotated dims, and ``sin`` already carrying the rotate_half sign:
``out[2i] = x[2i]*cos - x[2i+1]*sin``, ``out[2i+1] = x[2i+1]*cos + x[2i]*sin``.
"""
from __future__ import annotations

import math
from functools import lru_cache

import torch


def _lang_freqs(dim: int, theta: float = 10000.0) -> torch.Tensor:
    return 1.0 / (theta ** (torch.arange(0, dim, 2, dtype=torch.float64) / dim))


def _pixel_freqs(dim: int, max_freq: float = 10.0) -> torch.Tensor:
    return torch.logspace(0.0, math.log(max_freq / 2) / math.log(2), dim // 2, base=2, dtype=torch.float64) * math.pi


def _repeat2(f: torch.Tensor) -> torch.Tensor:
    return f.repeat_interleave(2, dim=-1)


@lru_cache(maxsize=16)
def rotary_angles(text_len: int, image_size: int, dim_head: int) -> torch.Tensor:
    """Angles (n+1, rotated_dims) in float64."""
    rot_dim = dim_head // 3
    img_len = image_size * image_size
    lang = _lang_freqs(rot_dim)
    pix = _pixel_freqs(rot_dim)

    text_pos = torch.cat([torch.arange(text_len, dtype=torch.float64), torch.full((img_len,), 8192.0, dtype=torch.float64)])
    text_freqs = _repeat2(text_pos[:, None] * lang[None, :])  # (T+I, 22)

    axial = torch.linspace(-1, 1, image_size, dtype=torch.float64)
    ax = _repeat2(axial[:, None] * pix[None, :])  # (S, 20)
    h = ax[:, None, :].expand(image_size, image_size, ax.shape[-1])
    w = ax[None, :, :].expand(image_size, image_size, ax.shape[-1])
    img_freqs = torch.cat([h, w], dim=-1).reshape(img_len, -1)  # (I, 40)
    text_axial = _repeat2(torch.full((text_len, 1), -10.0, dtype=torch.float64) * pix[None, :])
    text_axial = torch.cat([text_axial, text_axial], dim=-1)  # (T, 40)
    img_freqs = torch.cat([text_axial, img_freqs], dim=0)

    ang = torch.cat([text_freqs, img_freqs], dim=-1)
    assert ang.shape[-1] <= dim_head
    return ang


@lru_cache(maxsize=16)
def _tables_cpu(text_len: int, image_size: int, dim_head: int):
    ang = rotary_angles(text_len, image_size, dim_head)
    n1, r = ang.shape
    cos = torch.ones(n1, dim_head, dtype=torch.float64)
    sin = torch.zeros(n1, dim_head, dtype=torch.float64)
    cos[:, :r] = torch.cos(ang)
    s = torch.sin(ang)
    # fold rotate_half's sign: even lanes get -sin (x_even*cos - x_odd*sin), odd lanes +sin
    sign = torch.tensor([-1.0, 1.0], dtype=torch.float64).repeat(r // 2)
    sin[:, :r] = s * sign
    return cos.float().contiguous(), sin.float().contiguous()


def rotary_tables(text_len: int, image_size: int, dim_head: int, device=None):
    cos, sin = _tables_cpu(text_len, image_size, dim_head)
    if device is not None:
        cos, sin = cos.to(device), sin.to(device)
    return cos, sin


IMAGE_TEXT_POS = 8192.0   # the text position of every image token (rotary_angles)
TEXT_AXIAL_POS = -10.0    # the axial (row / column) position of every text token


@lru_cache(maxsize=16)
def _freq_split_cpu(dim_head: int):
    """The rotary frequencies per pair in revolutions per position unit, for angles computed in a kernel
    (the fused attention backward): (64,) fp32 = hi[32] + lo[32] with hi rounded to a 12-bit mantissa (so that
    position x hi is exact in fp32 for positions of <= 12 significant bits: text positions, 8192, -10) and lo the
    remainder; pairs [0, n_lang) turn with the text position, the next n_pix with the image row coordinate
    (linspace(-1, 1, S)), the next n_pix with the column coordinate, the rest (if any) not at all."""
    rot_dim = dim_head // 3
    f = torch.cat([_lang_freqs(rot_dim), _pixel_freqs(rot_dim), _pixel_freqs(rot_dim)]) / (2.0 * math.pi)
    n_lang, n_pix = _lang_freqs(rot_dim).numel(), _pixel_freqs(rot_dim).numel()
    assert f.numel() <= dim_head // 2 <= 32
    hi = torch.zeros(32, dtype=torch.float64)
    lo = torch.zeros(32, dtype=torch.float64)
    for j, v in enumerate(f.tolist()):
        m, e = math.frexp(v)
        h = math.ldexp(round(m * 4096.0) / 4096.0, e)
        hi[j], lo[j] = h, v - h
    return torch.cat([hi, lo]).float().contiguous(), n_lang, n_pix


def rotary_freq_split(dim_head: int, device=None):
    """``(rotf, n_lang, n_pix, image_text_pos, text_axial_pos)`` for ``attn_bwd_rope`` (see _freq_split_cpu)."""
    t, n_lang, n_pix = _freq_split_cpu(dim_head)
    return (t.to(device) if device is not None else t), n_lang, n_pix, IMAGE_TEXT_POS, TEXT_AXIAL_POS


def rotate_pairs(x: torch.Tensor) -> torch.Tensor:
    """(x0, x1) -> (x1, x0) on interleaved pairs (sign lives in the sin table)."""
    shp = x.shape
    x = x.reshape(*shp[:-1], shp[-1] // 2, 2).flip(-1)
    return x.reshape(shp)


def apply_rotary(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """x (..., n, D) with tables (n, D)."""
    return x * cos + rotate_pairs(x) * sin


def apply_rotary_inverse(g: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """Transpose (= inverse) of apply_rotary: used for the backward pass."""
    # y = x*c + P(x)*s  with P the pair swap  =>  x_grad = g*c + P(g*s)
    return g * cos + rotate_pairs(g * sin)
