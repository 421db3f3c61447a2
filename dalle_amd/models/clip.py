"""CLIP ViT-B/32 re-ranker for generated images (reference ``inference/run_inference.py:126,135-138``:
``_, logits_per_text = clip_model(images, clip.tokenize([query])); scores = logits_per_text[0].softmax(-1)``).

A native module with the OpenAI CLIP architecture and parameter names (``visual.conv1.weight``,
``visual.transformer.resblocks.{i}.attn.in_proj_weight``, ``token_embedding.weight``,
``text_projection``, ``logit_scale`` ...), so a converted OpenAI / open_clip state dict loads directly
with ``load_clip(path)`` (safetensors, or a plain ``torch.save`` state dict read with
``weights_only=True``; TorchScript archives are refused -- they cannot be loaded without executing
code). Without weights the model is random-init, which exercises the full re-ranking path but yields
meaningless scores (the CLI says so).

Preprocessing matches CLIP's: bicubic resize of the short side to 224, center crop, per-channel
normalisation -- done on the GPU on the decoder's output tensor instead of via PIL per image.
"""
from __future__ import annotations

import hashlib
import os
from collections import OrderedDict
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


@dataclass
class ClipConfig:
    embed_dim: int = 512
    image_resolution: int = 224
    vision_layers: int = 12
    vision_width: int = 768
    vision_patch_size: int = 32
    context_length: int = 77
    vocab_size: int = 49408
    transformer_width: int = 512
    transformer_heads: int = 8
    transformer_layers: int = 12


def vit_b32() -> ClipConfig:
    return ClipConfig()


class QuickGELU(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(1.702 * x)


class LayerNorm(nn.LayerNorm):
    """fp32 LayerNorm whatever the activation dtype (as in CLIP)."""

    def forward(self, x):
        return super().forward(x.float()).to(x.dtype)


class ResidualAttentionBlock(nn.Module):
    def __init__(self, width: int, heads: int, attn_mask: Optional[torch.Tensor] = None):
        super().__init__()
        self.attn = nn.MultiheadAttention(width, heads)
        self.ln_1 = LayerNorm(width)
        self.mlp = nn.Sequential(OrderedDict([("c_fc", nn.Linear(width, width * 4)), ("gelu", QuickGELU()),
                                              ("c_proj", nn.Linear(width * 4, width))]))
        self.ln_2 = LayerNorm(width)
        self.attn_mask = attn_mask

    def forward(self, x):  # (L, N, D)
        mask = None if self.attn_mask is None else self.attn_mask.to(dtype=x.dtype, device=x.device)
        h = self.ln_1(x)
        x = x + self.attn(h, h, h, need_weights=False, attn_mask=mask)[0]
        return x + self.mlp(self.ln_2(x))


class Transformer(nn.Module):
    def __init__(self, width: int, layers: int, heads: int, attn_mask: Optional[torch.Tensor] = None):
        super().__init__()
        self.resblocks = nn.Sequential(*[ResidualAttentionBlock(width, heads, attn_mask) for _ in range(layers)])

    def forward(self, x):
        return self.resblocks(x)


class VisionTransformer(nn.Module):
    def __init__(self, resolution: int, patch: int, width: int, layers: int, heads: int, output_dim: int):
        super().__init__()
        self.conv1 = nn.Conv2d(3, width, kernel_size=patch, stride=patch, bias=False)
        scale = width ** -0.5
        self.class_embedding = nn.Parameter(scale * torch.randn(width))
        self.positional_embedding = nn.Parameter(scale * torch.randn((resolution // patch) ** 2 + 1, width))
        self.ln_pre = LayerNorm(width)
        self.transformer = Transformer(width, layers, heads)
        self.ln_post = LayerNorm(width)
        self.proj = nn.Parameter(scale * torch.randn(width, output_dim))

    def forward(self, x):
        x = self.conv1(x)  # (B, W, g, g)
        x = x.flatten(2).transpose(1, 2)  # (B, g*g, W)
        cls = self.class_embedding.to(x.dtype).expand(x.shape[0], 1, -1)
        x = torch.cat([cls, x], dim=1) + self.positional_embedding.to(x.dtype)
        x = self.ln_pre(x).transpose(0, 1)
        x = self.transformer(x).transpose(0, 1)
        return self.ln_post(x[:, 0]) @ self.proj


class CLIP(nn.Module):
    def __init__(self, cfg: ClipConfig = None):
        super().__init__()
        cfg = cfg or vit_b32()
        self.cfg = cfg
        self.context_length = cfg.context_length
        self.visual = VisionTransformer(cfg.image_resolution, cfg.vision_patch_size, cfg.vision_width,
                                        cfg.vision_layers, cfg.vision_width // 64, cfg.embed_dim)
        mask = torch.full((cfg.context_length, cfg.context_length), float("-inf")).triu_(1)
        self.transformer = Transformer(cfg.transformer_width, cfg.transformer_layers, cfg.transformer_heads, mask)
        self.vocab_size = cfg.vocab_size
        self.token_embedding = nn.Embedding(cfg.vocab_size, cfg.transformer_width)
        self.positional_embedding = nn.Parameter(0.01 * torch.randn(cfg.context_length, cfg.transformer_width))
        self.ln_final = LayerNorm(cfg.transformer_width)
        self.text_projection = nn.Parameter(cfg.transformer_width ** -0.5 * torch.randn(cfg.transformer_width, cfg.embed_dim))
        self.logit_scale = nn.Parameter(torch.tensor(float(torch.log(torch.tensor(1 / 0.07)))))
        nn.init.normal_(self.token_embedding.weight, std=0.02)

    @property
    def dtype(self):
        return self.visual.conv1.weight.dtype

    def encode_image(self, image):
        return self.visual(image.to(self.dtype))

    def encode_text(self, text):
        x = self.token_embedding(text).to(self.dtype) + self.positional_embedding.to(self.dtype)
        x = self.transformer(x.transpose(0, 1)).transpose(0, 1)
        x = self.ln_final(x)
        # features at the end-of-text token (the highest id in each sequence)
        return x[torch.arange(x.shape[0], device=x.device), text.argmax(dim=-1)] @ self.text_projection

    def forward(self, image, text):
        img = self.encode_image(image)
        txt = self.encode_text(text)
        img = img / img.norm(dim=1, keepdim=True)
        txt = txt / txt.norm(dim=1, keepdim=True)
        logits_per_image = self.logit_scale.exp() * img.float() @ txt.float().t()
        return logits_per_image, logits_per_image.t()


# ------------------------------------------------------------------------------------------------
# preprocessing and tokenization
# ------------------------------------------------------------------------------------------------
def preprocess(images: torch.Tensor, resolution: int = 224) -> torch.Tensor:
    """images (B, 3, H, W) or (B, H, W, 3) in [0, 1] -> normalised (B, 3, R, R) CLIP input."""
    if images.shape[-1] == 3 and images.shape[1] != 3:
        images = images.permute(0, 3, 1, 2)
    x = images.float()
    h, w = x.shape[-2:]
    s = resolution / min(h, w)
    nh, nw = max(resolution, round(h * s)), max(resolution, round(w * s))
    x = F.interpolate(x, size=(nh, nw), mode="bicubic", align_corners=False, antialias=True).clamp_(0, 1)
    top, left = (nh - resolution) // 2, (nw - resolution) // 2
    x = x[..., top:top + resolution, left:left + resolution]
    mean = torch.tensor(CLIP_MEAN, device=x.device).view(1, 3, 1, 1)
    std = torch.tensor(CLIP_STD, device=x.device).view(1, 3, 1, 1)
    return (x - mean) / std


class ClipTokenizer:
    """CLIP's byte-level BPE when a HF ``tokenizer.json`` for it is available locally (``tokenizers``
    package); otherwise a deterministic word-hashing fallback with the same special ids
    (<|startoftext|> = 49406, <|endoftext|> = 49407) and context length."""

    SOT, EOT = 49406, 49407

    def __init__(self, path: Optional[str] = None, context_length: int = 77):
        self.context_length = context_length
        self._tok = None
        if path and os.path.exists(path):
            from tokenizers import Tokenizer

            self._tok = Tokenizer.from_file(path)

    def _ids(self, text: str) -> List[int]:
        if self._tok is not None:
            return self._tok.encode(text, add_special_tokens=False).ids
        out = []
        for w in text.lower().split():
            h = int.from_bytes(hashlib.blake2b(w.encode(), digest_size=4).digest(), "little")
            out.append(h % (self.SOT - 1) + 1)
        return out

    def __call__(self, texts: Sequence[str] | str) -> torch.Tensor:
        texts = [texts] if isinstance(texts, str) else list(texts)
        out = torch.zeros(len(texts), self.context_length, dtype=torch.long)
        for i, t in enumerate(texts):
            ids = [self.SOT] + self._ids(t)[: self.context_length - 2] + [self.EOT]
            out[i, : len(ids)] = torch.tensor(ids)
        return out


def load_clip(path: Optional[str] = None, device=None, dtype=torch.float32) -> CLIP:
    """CLIP ViT-B/32 with weights from ``path`` (safetensors / plain state dict), or random-init."""
    model = CLIP(vit_b32())
    if path:
        if path.endswith(".safetensors"):
            from safetensors.torch import load_file

            sd = load_file(path)
        else:
            try:
                sd = torch.load(path, map_location="cpu", weights_only=True)
            except Exception as e:  # noqa: BLE001
                raise RuntimeError(f"{path}: not a plain state dict (TorchScript CLIP archives are not loaded: "
                                   f"convert to safetensors first): {e}") from e
        sd = sd.get("state_dict", sd)
        sd = {k: v for k, v in sd.items() if k not in ("input_resolution", "context_length", "vocab_size")}
        model.load_state_dict(sd, strict=True)
    return model.to(device=device, dtype=dtype).eval()


@torch.no_grad()
def clip_scores(model: CLIP, tokenizer: ClipTokenizer, images: torch.Tensor, query: str) -> torch.Tensor:
    """Softmax over the images of CLIP's text->image logits (the reference's re-ranking score)."""
    dev = next(model.parameters()).device
    x = preprocess(images.to(dev)).to(model.dtype)
    text = tokenizer([query]).to(dev)
    _, logits_per_text = model(x, text)
    return logits_per_text[0].softmax(dim=-1)
