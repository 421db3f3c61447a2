"""The DALL-E text+image autoregressive transformer.

Module tree and parameter names follow the dalle-pytorch fork the reference pins
(``requirements.txt:2``) so checkpoints interchange:

  DALLE
  ├─ text_emb / image_emb        SharedEmbedding: row-slices of ``to_logits.1.weight`` (D10)
  ├─ transformer
  │   ├─ layers                  ReversibleSequence (``blocks.{i}.f.net`` / ``.g.net``)
  │   │                          or SequentialSequence (``layers.{i}.{0,1}``)
  │   │     LayerScale(.scale) -> PreNorm(.norm) -> PreShiftToken -> Attention / FeedForward
  │   └─ pos_emb                 rotary angles buffer
  └─ to_logits                   Sequential(LayerNorm, Linear(dim, total_tokens))

The module objects own the parameters; *execution* does not walk the wrapper chain: each residual
branch is one call into ``dalle_amd.ops`` (fused LayerNorm+shift, GEMM + rotary + sparse
attention + GEMM, GEMM + GEGLU + GEMM), which dispatches to the hand-written HIP kernels on
MI355X and to the pure-PyTorch reference on CPU.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..config import DALLEConfig
from .patterns import AttnGeometry
from .reversible import reversible_sequence
from .rotary import rotary_angles


def layer_scale_init(depth_index: int) -> float:
    """LayerScale init eps by 1-based layer index (D2)."""
    if depth_index <= 18:
        return 0.1
    if depth_index <= 24:
        return 1e-5
    return 1e-6


class Attention(nn.Module):
    """Sparse causal attention of one pattern type (D4-D6). Parameters: ``to_qkv``, ``to_out.0``."""

    def __init__(self, dim: int, heads: int, dim_head: int, attn_type: str):
        super().__init__()
        inner = heads * dim_head
        self.heads, self.dim_head, self.attn_type = heads, dim_head, attn_type
        self.to_qkv = nn.Linear(dim, inner * 3, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim), nn.Dropout(0.0))


class GEGLU(nn.Module):
    def forward(self, x):
        a, g = x.chunk(2, dim=-1)
        return a * F.gelu(g)


class FeedForward(nn.Module):
    """Linear(d, 2*mult*d) -> GEGLU -> Dropout(0) -> Linear(mult*d, d) (D9). Keys ``net.0``, ``net.3``."""

    def __init__(self, dim: int, mult: int = 4):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(dim, dim * mult * 2), GEGLU(), nn.Dropout(0.0), nn.Linear(dim * mult, dim))


class PreShiftToken(nn.Module):
    """Token shift wrapper (D8): parameterless, kept as a naming level (``.fn``)."""

    def __init__(self, fn: nn.Module, enabled: bool = True):
        super().__init__()
        self.fn = fn
        self.enabled = enabled


class PreNorm(nn.Module):
    def __init__(self, dim: int, fn: nn.Module):
        super().__init__()
        self.norm = nn.LayerNorm(dim)
        self.fn = fn


class LayerScale(nn.Module):
    def __init__(self, dim: int, depth_index: int, fn: nn.Module):
        super().__init__()
        self.scale = nn.Parameter(torch.full((1, 1, dim), layer_scale_init(depth_index)))
        self.fn = fn


class Deterministic(nn.Module):
    """Naming level of the reversible layout (``blocks.{i}.f.net``)."""

    def __init__(self, net: nn.Module):
        super().__init__()
        self.net = net


class ReversibleBlock(nn.Module):
    def __init__(self, f: nn.Module, g: nn.Module):
        super().__init__()
        self.f = Deterministic(f)
        self.g = Deterministic(g)


class ReversibleSequence(nn.Module):
    def __init__(self, blocks):
        super().__init__()
        self.blocks = nn.ModuleList([ReversibleBlock(f, g) for f, g in blocks])

    def pairs(self):
        return [(b.f.net, b.g.net) for b in self.blocks]


class SequentialSequence(nn.Module):
    def __init__(self, blocks):
        super().__init__()
        self.layers = nn.ModuleList([nn.ModuleList([f, g]) for f, g in blocks])

    def pairs(self):
        return [(l[0], l[1]) for l in self.layers]


class Transformer(nn.Module):
    def __init__(self, cfg: DALLEConfig):
        super().__init__()
        self.cfg = cfg
        self.geom = AttnGeometry(cfg.text_len, cfg.image_fmap_size, cfg.conv_kernel_size)
        shared_attn: Dict[str, tuple] = {}
        shared_ff: Dict[str, nn.Module] = {}
        blocks = []
        for ind, (attn_type, aid, fid) in enumerate(zip(cfg.attn_types, cfg.shared_attn_ids, cfg.shared_ff_ids)):
            key = str(aid)
            if key in shared_attn:
                attn, t = shared_attn[key]
                if t != attn_type:
                    raise ValueError(f"attn_types do not match shared_attn_ids (ind = {ind}, attn_type = {attn_type}, reused = {t})")
            else:
                attn = Attention(cfg.dim, cfg.heads, cfg.dim_head, attn_type)
                shared_attn[key] = (attn, attn_type)
            fkey = str(fid)
            ff = shared_ff.get(fkey)
            if ff is None:
                ff = FeedForward(cfg.dim, cfg.ff_mult)
                shared_ff[fkey] = ff
            f = LayerScale(cfg.dim, ind + 1, PreNorm(cfg.dim, PreShiftToken(attn, cfg.shift_tokens)))
            g = LayerScale(cfg.dim, ind + 1, PreNorm(cfg.dim, PreShiftToken(ff, cfg.shift_tokens)))
            blocks.append((f, g))
        self.layer_types = list(cfg.attn_types)
        self.layers = ReversibleSequence(blocks) if cfg.reversible else SequentialSequence(blocks)
        self.register_buffer("pos_emb", rotary_angles(cfg.text_len, cfg.image_fmap_size, cfg.dim_head).float()[None], persistent=True)

    # -- residual branches ------------------------------------------------------------------
    def _attn_out(self, ls: LayerScale, x: torch.Tensor) -> torch.Tensor:
        """attn(shift(LN(x))) before the LayerScale multiply."""
        pre: PreNorm = ls.fn
        attn: Attention = pre.fn.fn
        cfg = self.cfg
        h = ops.layernorm_shift(x, pre.norm.weight, pre.norm.bias, cfg.text_len, cfg.image_fmap_size, pre.fn.enabled)
        return ops.attention_block(h, attn.to_qkv.weight, attn.to_out[0].weight, attn.to_out[0].bias,
                                   attn.heads, self.geom, attn.attn_type)

    def _ff_out(self, ls: LayerScale, x: torch.Tensor) -> torch.Tensor:
        pre: PreNorm = ls.fn
        ff: FeedForward = pre.fn.fn
        cfg = self.cfg
        h = ops.layernorm_shift(x, pre.norm.weight, pre.norm.bias, cfg.text_len, cfg.image_fmap_size, pre.fn.enabled)
        return ops.feed_forward(h, ff.net[0].weight, ff.net[0].bias, ff.net[3].weight, ff.net[3].bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        pairs = self.layers.pairs()
        if self.cfg.reversible and ops.fused_reversible_available(x):
            cfg = self.cfg
            layers = []
            for f, g in pairs:
                pre, attn = f.fn, f.fn.fn.fn
                gpre, ff = g.fn, g.fn.fn.fn
                layers.append(((pre.norm.weight, pre.norm.bias, attn.to_qkv.weight, attn.to_out[0].weight, attn.to_out[0].bias,
                                f.scale, attn.heads, attn.attn_type, pre.fn.enabled),
                               (gpre.norm.weight, gpre.norm.bias, ff.net[0].weight, ff.net[0].bias, ff.net[3].weight,
                                ff.net[3].bias, g.scale, gpre.fn.enabled)))
            return ops.reversible_stack(x, layers, self.geom, cfg.text_len, cfg.image_fmap_size, cfg.reversible_recompute)
        if self.cfg.reversible:
            fns = [(lambda t, f=f: ops.scale_rows(self._attn_out(f, t), f.scale),
                    lambda t, g=g: ops.scale_rows(self._ff_out(g, t), g.scale)) for f, g in pairs]
            return reversible_sequence(x, fns)
        cfg = self.cfg
        if x.is_cuda:
            subs = []
            for f, g in pairs:
                pre, attn = f.fn, f.fn.fn.fn
                subs.append(("attn", ops.attn_meta(x, attn.to_qkv.weight, attn.heads, self.geom, attn.attn_type, pre.fn.enabled),
                             (pre.norm.weight, pre.norm.bias, attn.to_qkv.weight, attn.to_out[0].weight, attn.to_out[0].bias,
                              f.scale)))
                gpre, ff = g.fn, g.fn.fn.fn
                subs.append(("ff", ((cfg.text_len, cfg.image_fmap_size, bool(gpre.fn.enabled)),),
                             (gpre.norm.weight, gpre.norm.bias, ff.net[0].weight, ff.net[0].bias, ff.net[3].weight,
                              ff.net[3].bias, g.scale)))
            out = ops.sequential_stack(x, subs)
            if out is not None:
                return out
        for f, g in pairs:
            pre, attn = f.fn, f.fn.fn.fn
            x = ops.attn_sublayer(x, pre.norm.weight, pre.norm.bias, attn.to_qkv.weight, attn.to_out[0].weight,
                                  attn.to_out[0].bias, f.scale, attn.heads, self.geom, attn.attn_type, pre.fn.enabled)
            pre, ff = g.fn, g.fn.fn.fn
            x = ops.ff_sublayer(x, pre.norm.weight, pre.norm.bias, ff.net[0].weight, ff.net[0].bias, ff.net[3].weight,
                                ff.net[3].bias, g.scale, cfg.text_len, cfg.image_fmap_size, pre.fn.enabled)
        return x


class SharedEmbedding(nn.Module):
    """Embedding whose table is rows [start, end) of a Linear's weight (D10)."""

    def __init__(self, linear: nn.Linear, start_index: int, end_index: int):
        super().__init__()
        self.linear = linear
        self.start_index, self.end_index = start_index, end_index

    @property
    def weight(self):
        return self.linear.weight[self.start_index:self.end_index]

    def forward(self, ids):
        return F.embedding(ids, self.weight)


class DALLE(nn.Module):
    """DALL-E over VQGAN codes. ``forward(text, image, mask=None, return_loss=True)`` -> scalar loss."""

    def __init__(self, cfg: DALLEConfig, vae: Optional[nn.Module] = None):
        super().__init__()
        self.cfg = cfg
        self.num_text_tokens = cfg.total_text_tokens
        self.num_image_tokens = cfg.num_image_tokens
        self.text_seq_len = cfg.text_seq_len
        self.image_seq_len = cfg.image_seq_len
        self.total_tokens = cfg.total_tokens
        self.total_seq_len = cfg.seq_len
        self.loss_img_weight = cfg.loss_img_weight
        self.vae = vae
        self.transformer = Transformer(cfg)
        self.to_logits = nn.Sequential(nn.LayerNorm(cfg.dim), nn.Linear(cfg.dim, cfg.total_tokens))
        if cfg.share_input_output_emb:
            self.text_emb = SharedEmbedding(self.to_logits[1], 0, self.num_text_tokens)
            self.image_emb = SharedEmbedding(self.to_logits[1], self.num_text_tokens, self.total_tokens)
        else:
            self.text_emb = nn.Embedding(self.num_text_tokens, cfg.dim)
            self.image_emb = nn.Embedding(cfg.num_image_tokens, cfg.dim)

    # -- inputs -------------------------------------------------------------------------------
    def prepare_text(self, text: torch.Tensor) -> torch.Tensor:
        """K1: remap pad id 0 to a unique per-position id, prepend BOS=0."""
        assert text.shape[-1] == self.text_seq_len, f"text must be {self.text_seq_len} tokens"
        rng = torch.arange(self.text_seq_len, device=text.device) + (self.num_text_tokens - self.text_seq_len)
        text = torch.where(text == 0, rng, text)
        return F.pad(text, (1, 0), value=0)

    def embed(self, text_bos: torch.Tensor, image: Optional[torch.Tensor]) -> torch.Tensor:
        tokens = self.text_emb(text_bos)
        if image is not None and image.numel() > 0:
            tokens = torch.cat([tokens, self.image_emb(image)], dim=1)
        if tokens.shape[1] > self.total_seq_len:
            tokens = tokens[:, :-1]
        return tokens

    def forward(self, text, image=None, mask=None, return_loss: bool = False):
        """``mask`` is accepted for API parity and ignored, as in the pinned fork."""
        text_bos = self.prepare_text(text)
        if image is not None and image.dim() == 4:
            assert self.vae is not None, "raw images need a VAE"
            image = self.vae.get_codebook_indices(image)
        ops.begin_forward()
        x = None
        if self.cfg.share_input_output_emb and image is not None and image.numel() > 0:
            # one HIP gather kernel for pad remap + BOS + both tied tables, straight into the fp32 stream
            x = ops.embed_tokens(text, image, self.to_logits[1].weight, self.num_text_tokens - self.text_seq_len,
                                 self.num_text_tokens)
        if x is None:
            tokens = self.embed(text_bos, image)
            # fp32 residual stream, bf16 (or input dtype) compute inside the branches
            x = tokens.float() if tokens.is_cuda else tokens
        out = self.transformer(x)
        norm, head = self.to_logits[0], self.to_logits[1]
        if not return_loss:
            h = F.layer_norm(out, (out.shape[-1],), norm.weight, norm.bias)
            return ops.reference.masked_logits(h.to(head.weight.dtype), head.weight, head.bias, self.text_seq_len, self.num_text_tokens)
        assert image is not None, "when training, image must be supplied"
        labels = torch.cat([text_bos[:, 1:], image + self.num_text_tokens], dim=1)
        return ops.logits_loss(out, norm.weight, norm.bias, head.weight, head.bias, labels,
                               self.text_seq_len, self.num_text_tokens, self.loss_img_weight)

    # -- generation (D11) -------------------------------------------------------------------------
    @torch.no_grad()
    def generate_images(self, text, *, clip=None, mask=None, filter_thres=None, temperature: float = 1.0, img=None,
                        num_init_img_tokens=None, top_k: int = 0, top_p: float = 1.0, use_cache: bool = True,
                        return_codes: bool = False, use_graph=None):
        """Sample 1024 image tokens per caption with the KV-cache decoder (hipGraph-replayed on MI355X)
        and decode them with ``self.vae`` to (b, 3, H, W) images in [0, 1] (codes if no VAE)."""
        from .generation import make_decode_engine

        if filter_thres is not None and not top_k:
            top_k = max(1, int((1 - filter_thres) * self.num_image_tokens))
        text_bos = self.prepare_text(text)
        eng = getattr(self, "_decode_engine", None)
        if eng is None or eng.B != text.shape[0] or eng.device != text.device:
            eng = make_decode_engine(self, text.shape[0], device=text.device)
            self._decode_engine = eng
        codes = eng.generate(text_bos, temperature=temperature, top_k=top_k, top_p=top_p, use_graph=use_graph)
        if return_codes or self.vae is None:
            return codes
        return self.vae.decode(codes)

    # -- checkpoint helpers --------------------------------------------------------------------
    def unique_parameters(self) -> List[nn.Parameter]:
        return list(self.parameters())
