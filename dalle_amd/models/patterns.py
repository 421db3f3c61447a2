"""Sparse attention patterns -- the single source of truth for training masks, the HIP
kernels' block schedules and the decode-time static masks.

Semantics reproduced (dalle-pytorch fork, [ext], anchored at ``task.py:63-64`` and
``inference/run_inference.py:72``):

* A sequence of ``n = text_len + image_seq_len - 1`` tokens: ``text_len = 1 + text_seq_len`` text
  positions (BOS + text), then the image tokens in raster order (the last image token is dropped).
* Text queries attend causally to text keys.
* Image queries attend to *all* text keys plus a pattern-specific set of earlier image keys
  inside one joint softmax:
    - ``axial_row``: same image row, column <= own column
    - ``axial_col``: same image column, row <= own row
    - ``conv_like``: the upper-left ``k x k`` window (incl. self), rows r-k+1..r, cols c-k+1..c
    - ``full``:      every earlier token (dense causal)

The MI355X kernels use a *padded storage layout* for q/k/v: text rows ``[0, text_len)`` padded to
``text_pad = ceil32(text_len)`` rows, followed by the ``image_seq_len`` image rows (the padded last
image token included). For ``axial_col`` layers the image rows are stored column-major, which turns
column attention into row attention over contiguous keys.
"""
from __future__ import annotations

from dataclasses import dataclass
from functools import lru_cache

import torch

PATTERN_IDS = {"full": 0, "axial_row": 1, "axial_col": 2, "conv_like": 3}


@dataclass(frozen=True)
class AttnGeometry:
    text_len: int       # BOS + text tokens (257)
    image_size: int     # image token grid side (32)
    kernel_size: int = 5  # conv_like window

    @property
    def image_seq_len(self) -> int:
        return self.image_size * self.image_size

    @property
    def seq_len(self) -> int:
        """Unpadded model sequence length n (1280)."""
        return self.text_len + self.image_seq_len - 1

    @property
    def text_pad(self) -> int:
        return (self.text_len + 31) // 32 * 32

    @property
    def padded_len(self) -> int:
        """Rows of the padded q/k/v storage layout (1312)."""
        return self.text_pad + self.image_seq_len


def allowed(geom: AttnGeometry, attn_type: str, i: torch.Tensor, j: torch.Tensor) -> torch.Tensor:
    """Boolean mask: may query at sequence position ``i`` attend key at sequence position ``j``."""
    T, S = geom.text_len, geom.image_size
    causal = j <= i
    key_text = j < T
    q_img = i >= T
    qk = (i - T).clamp(min=0)
    kk = (j - T).clamp(min=0)
    qr, qc = qk // S, qk % S
    kr, kc = kk // S, kk % S
    if attn_type == "full":
        local = torch.ones_like(causal)
    elif attn_type == "axial_row":
        local = (qr == kr) & (kc <= qc)
    elif attn_type == "axial_col":
        local = (qc == kc) & (kr <= qr)
    elif attn_type == "conv_like":
        K = geom.kernel_size
        local = (kr <= qr) & (kr > qr - K) & (kc <= qc) & (kc > qc - K)
    else:
        raise ValueError(attn_type)
    img_rule = key_text | ((~key_text) & local)
    return causal & torch.where(q_img, img_rule, key_text)


@lru_cache(maxsize=64)
def _static_mask_cpu(geom: AttnGeometry, attn_type: str, n: int) -> torch.Tensor:
    i = torch.arange(n).view(n, 1)
    j = torch.arange(n).view(1, n)
    return allowed(geom, attn_type, i, j)


@lru_cache(maxsize=64)
def _static_mask_dev(geom: AttnGeometry, attn_type: str, n: int, device: str) -> torch.Tensor:
    return _static_mask_cpu(geom, attn_type, n).to(device)


def static_mask(geom: AttnGeometry, attn_type: str, n: int | None = None, device=None) -> torch.Tensor:
    """Dense (n, n) boolean mask (True = attend) -- the inference / golden-test form (D6). Cached per device (read-only:
    the caption prefill asks for it in every layer, and a 1.6 MB pageable host copy each time cost most of its time)."""
    n = geom.seq_len if n is None else n
    if device is None:
        return _static_mask_cpu(geom, attn_type, n)
    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return _static_mask_dev(geom, attn_type, n, str(dev))


def storage_index(geom: AttnGeometry, attn_type: str) -> torch.Tensor:
    """Padded-layout storage row for every sequence position 0..n (n+1 entries, the padding token incl.)."""
    T, S, Tp = geom.text_len, geom.image_size, geom.text_pad
    n1 = geom.seq_len + 1
    p = torch.arange(n1)
    k = (p - T).clamp(min=0)
    if attn_type == "axial_col":
        k_st = (k % S) * S + k // S
    else:
        k_st = k
    return torch.where(p < T, p, Tp + k_st)


def local_key_window(geom: AttnGeometry, attn_type: str):
    """For image queries: how many whole image rows before the query's row the local keys reach."""
    if attn_type in ("axial_row", "axial_col"):
        return 0
    if attn_type == "conv_like":
        return geom.kernel_size - 1
    return None  # full: all earlier rows
