"""VQGAN decoder on the hand-written HIP kernels (``csrc/kernels/conv.hip``).

Runs the taming ``Decoder`` of :mod:`dalle_amd.models.vqgan` with NHWC bf16 activations:

* every 3x3 convolution is the implicit-GEMM MFMA kernel (``conv3x3``); a ResNet block is
  ``gn_stats -> conv3x3(GN+SiLU fused into its input gather) -> gn_stats -> conv3x3(GN+SiLU in,
  residual out)``, and the Upsample's 2x nearest interpolation is folded into its conv's gather;
* the 1x1 convolutions (``post_quant_conv``, the ``nin_shortcut`` of channel-changing blocks, the
  attention block's q/k/v/proj) are plain GEMMs over the NHWC pixels (hipBLASLt);
* the 32x32 attention block: ``gn_apply`` -> one qkv GEMM -> scores (fp32) -> ``softmax_rows`` ->
  P V -> proj + residual;
* ``conv_out``: final GroupNorm + SiLU + 3x3 conv to RGB + clamp / rescale, written as NCHW fp32.

Weights are converted once (bf16, conv kernels as [Cout, 3*3*Cin] tap-major / channel-contiguous) and
cached on the module; the fp32 torch ``Decoder`` stays the numerics reference
(``tests/test_vqgan_gpu.py``).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import os

import torch
import torch.nn.functional as F

from .vqgan import AttnBlock, Decoder, ResnetBlock, Upsample


def _conv_w(conv: torch.nn.Conv2d) -> torch.Tensor:
    w = conv.weight.detach()
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).to(torch.bfloat16).contiguous()


def _lin_w(conv: torch.nn.Conv2d) -> torch.Tensor:
    return conv.weight.detach().reshape(conv.weight.shape[0], -1).to(torch.bfloat16).contiguous()


def _f32(t: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
    return None if t is None else t.detach().float().contiguous()


# GroupNorm + SiLU as a separate bf16 pass ahead of the 3x3 conv for images of at least this many pixels (default 0:
# every GN conv; batch 64 decoder 45.0 -> 42.1 ms, the gain at the low-resolution / high-channel levels, neutral at
# 256 x 256: profiles/r6_vqgan_conv_out.txt). DALLE_AMD_VQGAN_GN_PREPASS=<pixels> keeps smaller images on the
# fused-gather form.
_GN_PREPASS_MIN_HW = int(os.environ.get("DALLE_AMD_VQGAN_GN_PREPASS", "0"))


class HipDecoder:
    """Executes ``post_quant_conv`` + ``decoder`` of a :class:`VQGanVAE` on MI355X."""

    def __init__(self, post_quant_conv: torch.nn.Conv2d, decoder: Decoder):
        from ..ops.ext import load_extension

        self.C = load_extension(required=True)
        self.dec = decoder
        self.pq = (_lin_w(post_quant_conv), _f32(post_quant_conv.bias))
        self._w: Dict[int, tuple] = {}

    # -- cached weights ------------------------------------------------------------------------
    def _gn(self, gn: torch.nn.GroupNorm):
        return _f32(gn.weight), _f32(gn.bias), float(gn.eps)

    def _cached(self, key, build):
        if key not in self._w:
            self._w[key] = build()
        return self._w[key]

    # -- blocks --------------------------------------------------------------------------------
    def conv3x3(self, x, conv, gn=None, res=None, ups=False):
        w, b = self._cached(id(conv), lambda: (_conv_w(conv), _f32(conv.bias)))
        if gn is None:
            return self.C.conv3x3(x, w, b, res, ups=ups)
        gamma, beta, eps = self._cached(id(gn), lambda: self._gn(gn))
        mean, rstd = self.C.gn_stats(x, eps)
        if x.shape[1] * x.shape[2] >= _GN_PREPASS_MIN_HW:
            # SiLU(GN(x)) once per element into bf16, then the plain conv: the fused form applies it in the gather,
            # i.e. 9 times per element (once per tap)
            return self.C.conv3x3(self.C.gn_apply(x, mean, rstd, gamma, beta, silu=True), w, b, res, ups=ups)
        return self.C.conv3x3(x, w, b, res, mean, rstd, gamma, beta, ups=ups)

    def linear(self, x, conv):
        """1x1 conv over NHWC pixels: (N, H, W, Cin) -> (N, H, W, Cout) (+ bias), one GEMM."""
        w, b = self._cached(id(conv), lambda: (_lin_w(conv), _f32(conv.bias)))
        n, h, wd, c = x.shape
        y = torch.mm(x.view(-1, c), w.t())
        if b is not None:
            y.add_(b.to(y.dtype))
        return y.view(n, h, wd, -1)

    def resblock(self, x, blk: ResnetBlock):
        h = self.conv3x3(x, blk.conv1, gn=blk.norm1)
        sc = x if blk.nin_shortcut is None else self.linear(x, blk.nin_shortcut)
        return self.conv3x3(h, blk.conv2, gn=blk.norm2, res=sc.contiguous())

    def attn(self, x, blk: AttnBlock):
        n, hh, ww, c = x.shape
        gamma, beta, eps = self._cached(id(blk.norm), lambda: self._gn(blk.norm))
        mean, rstd = self.C.gn_stats(x, eps)
        hn = self.C.gn_apply(x, mean, rstd, gamma, beta)
        wqkv, bqkv = self._cached(("qkv", id(blk)), lambda: (
            torch.cat([_lin_w(blk.q), _lin_w(blk.k), _lin_w(blk.v)]).contiguous(),
            torch.cat([_f32(blk.q.bias), _f32(blk.k.bias), _f32(blk.v.bias)]).contiguous()))
        qkv = torch.addmm(bqkv.to(torch.bfloat16), hn.view(-1, c), wqkv.t()).view(n, hh * ww, 3, c)
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        s = torch.bmm(q, k.transpose(1, 2), out_dtype=torch.float32)
        p = self.C.softmax_rows(s, float(c) ** -0.5)
        o = torch.bmm(p, v)
        return x + self.linear(o.view(n, hh, ww, c), blk.proj_out)

    # -- whole decoder -------------------------------------------------------------------------
    @torch.no_grad()
    def __call__(self, z_nhwc: torch.Tensor) -> torch.Tensor:
        """z (N, h, w, z_channels) bf16 -> images (N, 3, H, W) fp32 in [0, 1]."""
        d = self.dec
        n, hh, ww, c = z_nhwc.shape
        wpq, bpq = self.pq
        x = torch.addmm(bpq.to(torch.bfloat16), z_nhwc.reshape(-1, c), wpq.t()).view(n, hh, ww, -1)
        x = self.conv3x3(x.contiguous(), d.conv_in)
        x = self.resblock(x, d.mid.block_1)
        x = self.attn(x, d.mid.attn_1)
        x = self.resblock(x, d.mid.block_2)
        for i_level in reversed(range(d.num_resolutions)):
            up = d.up[i_level]
            for i_block in range(d.num_res_blocks + 1):
                x = self.resblock(x, up.block[i_block])
                if len(up.attn) > 0:
                    x = self.attn(x, up.attn[i_block])
            if i_level != 0:
                x = self.conv3x3(x, up.upsample.conv, ups=True)
        gamma, beta, eps = self._cached(id(d.norm_out), lambda: self._gn(d.norm_out))
        mean, rstd = self.C.gn_stats(x, eps)
        wout, bout = self._cached(id(d.conv_out), lambda: (_conv_w(d.conv_out), _f32(d.conv_out.bias)))
        return self.C.conv_out(x, wout, bout, mean, rstd, gamma, beta)


def supported(decoder: Decoder) -> bool:
    """The HIP path needs channel counts the kernels tile (multiples of 128 for the 3x3 convs, <= 128
    channels into the RGB conv) and 32-group GroupNorms."""
    convs: List[torch.nn.Conv2d] = [m for m in decoder.modules() if isinstance(m, torch.nn.Conv2d) and m.kernel_size == (3, 3)]
    for m in convs:
        if m is decoder.conv_out:
            continue
        if m.in_channels % 64 or m.out_channels % 128:
            return False
    return decoder.conv_out.in_channels <= 128 and decoder.conv_out.in_channels % 32 == 0
