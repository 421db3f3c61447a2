"""VQGAN (taming-transformers) encoder + decoder.

``VQGanVAE(ckpt_path, config_path)``: ``decode(seq)`` = codebook embed (HIP gather kernel on MI355X,
``one_hot(seq) @ codebook``) -> ``post_quant_conv`` -> conv decoder (ResNet blocks, GroupNorm,
swish, nearest x2 upsampling, attention at the 32x32 resolution) -> ``(clamp(-1,1)+1)/2``.
``get_codebook_indices(img)`` (dalle-pytorch's API; training uses precomputed LAION codes) runs the
conv encoder (stride-2 downsampling, same blocks) -> ``quant_conv`` -> code selection: the Gumbel
quantizer's ``proj`` logits (argmax = the mode; ``gumbel_tau`` > 0 samples like taming's eval-time
``gumbel_softmax(hard=True)``), or the nearest codebook vector for a plain VQ checkpoint.
Parameter names follow taming's ``VQModel`` / ``GumbelVQ`` so a real checkpoint's state dict loads
(``torch.load(weights_only=True)``); without a checkpoint the decoder is random-init (benchmarks).
Default config = the LAION ``vqgan_gumbel_f8`` one: 8192 codes x 256 dims, ch 128, ch_mult
(1,1,2,4), 2 res blocks, attention at 32.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F


def Normalize(c):
    return nn.GroupNorm(num_groups=32, num_channels=c, eps=1e-6, affine=True)


class ResnetBlock(nn.Module):
    def __init__(self, in_channels, out_channels=None):
        super().__init__()
        out_channels = out_channels or in_channels
        self.norm1 = Normalize(in_channels)
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, 1, 1)
        self.norm2 = Normalize(out_channels)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, 1, 1)
        self.nin_shortcut = nn.Conv2d(in_channels, out_channels, 1) if in_channels != out_channels else None

    def forward(self, x):
        h = self.conv1(F.silu(self.norm1(x)))
        h = self.conv2(F.silu(self.norm2(h)))
        if self.nin_shortcut is not None:
            x = self.nin_shortcut(x)
        return x + h


class AttnBlock(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.norm = Normalize(c)
        self.q, self.k, self.v = nn.Conv2d(c, c, 1), nn.Conv2d(c, c, 1), nn.Conv2d(c, c, 1)
        self.proj_out = nn.Conv2d(c, c, 1)

    def forward(self, x):
        h = self.norm(x)
        b, c, hh, ww = h.shape
        q = self.q(h).reshape(b, c, hh * ww).transpose(1, 2)
        k = self.k(h).reshape(b, c, hh * ww).transpose(1, 2)
        v = self.v(h).reshape(b, c, hh * ww).transpose(1, 2)
        o = F.scaled_dot_product_attention(q[:, None], k[:, None], v[:, None])[:, 0]
        return x + self.proj_out(o.transpose(1, 2).reshape(b, c, hh, ww))


class Upsample(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 1, 1)

    def forward(self, x):
        return self.conv(F.interpolate(x, scale_factor=2.0, mode="nearest"))


class Downsample(nn.Module):
    """3x3 stride-2 conv with taming's asymmetric (0, 1, 0, 1) zero padding."""

    def __init__(self, c):
        super().__init__()
        self.conv = nn.Conv2d(c, c, 3, 2, 0)

    def forward(self, x):
        return self.conv(F.pad(x, (0, 1, 0, 1)))


class Encoder(nn.Module):
    def __init__(self, *, ch=128, in_channels=3, ch_mult: Sequence[int] = (1, 1, 2, 4), num_res_blocks=2,
                 attn_resolutions: Sequence[int] = (32,), resolution=256, z_channels=256, double_z=False, **ignore):
        super().__init__()
        self.num_resolutions = len(ch_mult)
        self.num_res_blocks = num_res_blocks
        self.conv_in = nn.Conv2d(in_channels, ch, 3, 1, 1)
        curr_res = resolution
        in_mult = (1,) + tuple(ch_mult)
        self.down = nn.ModuleList()
        block_in = ch
        for i_level in range(self.num_resolutions):
            block, attn = nn.ModuleList(), nn.ModuleList()
            block_in, block_out = ch * in_mult[i_level], ch * ch_mult[i_level]
            for _ in range(num_res_blocks):
                block.append(ResnetBlock(block_in, block_out))
                block_in = block_out
                if curr_res in attn_resolutions:
                    attn.append(AttnBlock(block_in))
            down = nn.Module()
            down.block, down.attn = block, attn
            if i_level != self.num_resolutions - 1:
                down.downsample = Downsample(block_in)
                curr_res //= 2
            self.down.append(down)
        self.mid = nn.Module()
        self.mid.block_1 = ResnetBlock(block_in, block_in)
        self.mid.attn_1 = AttnBlock(block_in)
        self.mid.block_2 = ResnetBlock(block_in, block_in)
        self.norm_out = Normalize(block_in)
        self.conv_out = nn.Conv2d(block_in, 2 * z_channels if double_z else z_channels, 3, 1, 1)

    def forward(self, x):
        h = self.conv_in(x)
        for i_level in range(self.num_resolutions):
            down = self.down[i_level]
            for i_block in range(self.num_res_blocks):
                h = down.block[i_block](h)
                if len(down.attn) > 0:
                    h = down.attn[i_block](h)
            if i_level != self.num_resolutions - 1:
                h = down.downsample(h)
        h = self.mid.block_2(self.mid.attn_1(self.mid.block_1(h)))
        return self.conv_out(F.silu(self.norm_out(h)))


class Decoder(nn.Module):
    def __init__(self, *, ch=128, out_ch=3, ch_mult: Sequence[int] = (1, 1, 2, 4), num_res_blocks=2,
                 attn_resolutions: Sequence[int] = (32,), resolution=256, z_channels=256, **ignore):
        super().__init__()
        self.num_resolutions = len(ch_mult)
        self.num_res_blocks = num_res_blocks
        block_in = ch * ch_mult[-1]
        curr_res = resolution // 2 ** (self.num_resolutions - 1)
        self.conv_in = nn.Conv2d(z_channels, block_in, 3, 1, 1)
        self.mid = nn.Module()
        self.mid.block_1 = ResnetBlock(block_in, block_in)
        self.mid.attn_1 = AttnBlock(block_in)
        self.mid.block_2 = ResnetBlock(block_in, block_in)
        self.up = nn.ModuleList()
        for i_level in reversed(range(self.num_resolutions)):
            block, attn = nn.ModuleList(), nn.ModuleList()
            block_out = ch * ch_mult[i_level]
            for _ in range(num_res_blocks + 1):
                block.append(ResnetBlock(block_in, block_out))
                block_in = block_out
                if curr_res in attn_resolutions:
                    attn.append(AttnBlock(block_in))
            up = nn.Module()
            up.block, up.attn = block, attn
            if i_level != 0:
                up.upsample = Upsample(block_in)
                curr_res *= 2
            self.up.insert(0, up)
        self.norm_out = Normalize(block_in)
        self.conv_out = nn.Conv2d(block_in, out_ch, 3, 1, 1)

    def forward(self, z):
        h = self.conv_in(z)
        h = self.mid.block_2(self.mid.attn_1(self.mid.block_1(h)))
        for i_level in reversed(range(self.num_resolutions)):
            up = self.up[i_level]
            for i_block in range(self.num_res_blocks + 1):
                h = up.block[i_block](h)
                if len(up.attn) > 0:
                    h = up.attn[i_block](h)
            if i_level != 0:
                h = up.upsample(h)
        return self.conv_out(F.silu(self.norm_out(h)))


class GumbelQuantize(nn.Module):
    """Codebook (``embed``) + the Gumbel quantizer's logit projection (``proj``; plain VQ: None)."""

    def __init__(self, n_embed: int, embedding_dim: int, num_hiddens: Optional[int] = None):
        super().__init__()
        self.embed = nn.Embedding(n_embed, embedding_dim)
        self.proj = nn.Conv2d(num_hiddens, n_embed, 1) if num_hiddens is not None else None


class VQGanVAE(nn.Module):
    def __init__(self, vqgan_model_path: Optional[str] = None, vqgan_config_path: Optional[str] = None, *,
                 n_embed: int = 8192, embed_dim: int = 256, ddconfig: Optional[dict] = None, is_gumbel: bool = True):
        super().__init__()
        if vqgan_config_path is not None:
            import yaml

            with open(vqgan_config_path) as f:
                conf = yaml.load(f, Loader=yaml.SafeLoader)
            params = conf["model"]["params"]
            ddconfig = params["ddconfig"]
            n_embed, embed_dim = params["n_embed"], params["embed_dim"]
            is_gumbel = "Gumbel" in conf["model"].get("target", "GumbelVQ")
        ddconfig = ddconfig or dict(ch=128, out_ch=3, ch_mult=(1, 1, 2, 4), num_res_blocks=2, attn_resolutions=(32,),
                                    resolution=256, z_channels=256)
        self.encoder = Encoder(**ddconfig)
        self.quant_conv = nn.Conv2d(ddconfig["z_channels"], embed_dim, 1)
        self.decoder = Decoder(**ddconfig)
        self.post_quant_conv = nn.Conv2d(embed_dim, ddconfig["z_channels"], 1)
        self.quantize = GumbelQuantize(n_embed, embed_dim, embed_dim if is_gumbel else None)
        self.is_gumbel = is_gumbel
        self.num_tokens = n_embed
        self.num_layers = len(ddconfig["ch_mult"]) - 1
        self.image_size = ddconfig["resolution"]
        if vqgan_model_path is not None:
            sd = torch.load(vqgan_model_path, map_location="cpu", weights_only=True)
            sd = sd.get("state_dict", sd)
            if "quantize.embedding.weight" in sd:  # plain VectorQuantizer naming
                sd = dict(sd, **{"quantize.embed.weight": sd["quantize.embedding.weight"]})
            keep = ("encoder.", "quant_conv.", "decoder.", "post_quant_conv.", "quantize.embed.", "quantize.proj.")
            missing, _ = self.load_state_dict({k: v for k, v in sd.items() if k.startswith(keep)}, strict=False)
            needed = [k for k in missing if not k.startswith(("encoder.", "quant_conv.", "quantize.proj."))]
            if needed:
                raise RuntimeError(f"VQGAN checkpoint is missing decoder weights: {needed[:5]}")
            self.has_encoder = not any(k.startswith(("encoder.", "quant_conv.")) for k in missing)

    @property
    def codebook(self) -> torch.Tensor:
        return self.quantize.embed.weight

    def embed_codes(self, seq: torch.Tensor) -> torch.Tensor:
        b, n = seq.shape
        side = int(round(n ** 0.5))
        cb = self.codebook
        if seq.is_cuda and cb.dtype == torch.float32:
            from ..ops.ext import load_extension

            return load_extension(required=True).vq_embed(seq.contiguous().long(), cb.detach().contiguous(), side)
        z = F.one_hot(seq, num_classes=self.num_tokens).to(cb.dtype) @ cb
        return z.view(b, side, side, -1).permute(0, 3, 1, 2).contiguous()

    @torch.no_grad()
    def decode(self, img_seq: torch.Tensor) -> torch.Tensor:
        if img_seq.is_cuda and self.use_hip_decoder():
            # K20 on the hand-written HIP kernels (models/vqgan_hip.py): NHWC bf16 from the codebook gather on
            hip = self._hip_decoder
            b, n = img_seq.shape
            side = int(round(n ** 0.5))
            cb = self._codebook_bf16()
            z = F.embedding(img_seq.long(), cb).view(b, side, side, cb.shape[1])
            return hip(z)
        z = self.embed_codes(img_seq)
        img = self.decoder(self.post_quant_conv(z))
        return (img.clamp(-1.0, 1.0) + 1) * 0.5

    hip_decoder = True  # False: the PyTorch / MIOpen decoder (numerics A/B in tests/test_vqgan_gpu.py)

    def use_hip_decoder(self) -> bool:
        """True when the decoder runs on the HIP kernels (MI355X, supported channel layout, ``hip_decoder``)."""
        if not self.hip_decoder:
            return False
        if getattr(self, "_hip_decoder", None) is None:
            from .vqgan_hip import HipDecoder, supported

            if not supported(self.decoder):
                return False
            self._hip_decoder = HipDecoder(self.post_quant_conv, self.decoder)
        return True

    def _codebook_bf16(self) -> torch.Tensor:
        cb = self.codebook
        key = (cb.data_ptr(), cb._version)
        if getattr(self, "_cb_key", None) != key:
            self._cb_bf16 = cb.detach().to(torch.bfloat16).contiguous()
            self._cb_key = key
        return self._cb_bf16

    @torch.no_grad()
    def get_codebook_indices(self, images: torch.Tensor, gumbel_tau: float = 0.0, generator=None) -> torch.Tensor:
        """(B, 3, H, W) images in [0, 1] -> (B, (H/f)^2) code indices (dalle-pytorch ``VQGanVAE`` API)."""
        if not getattr(self, "has_encoder", True):
            raise RuntimeError("this VQGAN checkpoint holds no encoder weights")
        h = self.quant_conv(self.encoder(2 * images - 1))
        if self.quantize.proj is not None:
            logits = self.quantize.proj(h)
            if gumbel_tau > 0:
                u = torch.rand(logits.shape, device=logits.device, generator=generator).clamp_(1e-20, 1.0)
                logits = logits / gumbel_tau - torch.log(-torch.log(u))
            idx = logits.argmax(dim=1)
        else:
            z = h.permute(0, 2, 3, 1).reshape(-1, h.shape[1])
            cb = self.codebook.to(z.dtype)
            d = (z * z).sum(1, keepdim=True) - 2 * z @ cb.t() + (cb * cb).sum(1)[None]
            idx = d.argmin(dim=1).view(h.shape[0], h.shape[2], h.shape[3])
        return idx.flatten(1)
