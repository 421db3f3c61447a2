"""Autoregressive text->image decoding with a KV cache (BASELINE config 5).

One decode step pushes ONE position through every layer: fused LayerNorm + cached token shift
(per-branch LN history), QKV GEMM, rotary into the KV cache, sparse decode attention over only the
keys the layer's static pattern allows (text prefix + row / column / 5x5 window), output GEMM,
LayerScale residual, then the final norm, the image-vocabulary head and sampling (temperature,
top-k, top-p, Gumbel-max). Every positional quantity is read from a device scalar, so on MI355X the
whole step is captured ONCE into a hipGraph and replayed for each of the 1024 image tokens.

The CPU path runs the same step with the reference ops (tests compare it against the full forward).
"""
from __future__ import annotations

import math
import os
import threading
from typing import List, Optional

import torch
import torch.nn.functional as F

from .patterns import PATTERN_IDS, static_mask
from .rotary import apply_rotary, rotary_tables

# hipGraph captures of different engines (e.g. one serving generator per GPU, each in its own thread)
# run one at a time, in thread-local capture mode: another thread's replays and allocations on its own
# device neither break a capture nor are refused while it runs
_CAPTURE_LOCK = threading.Lock()


def filter_logits(logits: torch.Tensor, top_k: int = 0, top_p: float = 1.0) -> torch.Tensor:
    """K18: top-k then nucleus filtering (fill -inf); graph-capturable (no host sync)."""
    if top_k and top_k > 0:
        kth = torch.topk(logits, min(top_k, logits.shape[-1]), dim=-1).values[..., -1:]
        logits = logits.masked_fill(logits < kth, float("-inf"))
    if top_p is not None and top_p < 1.0:
        sorted_logits, sorted_idx = torch.sort(logits, descending=True, dim=-1)
        cum = torch.softmax(sorted_logits, dim=-1).cumsum(-1)
        remove = cum - torch.softmax(sorted_logits, dim=-1) > top_p  # keep the token that crosses top_p
        sorted_logits = sorted_logits.masked_fill(remove, float("-inf"))
        logits = torch.full_like(logits, float("-inf")).scatter(-1, sorted_idx, sorted_logits)
    return logits


def gumbel_sample(logits: torch.Tensor, temperature: float = 1.0, generator=None) -> torch.Tensor:
    u = torch.rand(logits.shape, device=logits.device, generator=generator).clamp_(1e-20, 1.0)
    return torch.argmax(logits / max(temperature, 1e-10) - torch.log(-torch.log(u)), dim=-1)


class DecodeEngine:
    def __init__(self, model, batch_size: int, device=None, use_hip: Optional[bool] = None, skinny: bool = True,
                 partials: int = 2, fused_sampler: bool = True, ln_tail: Optional[bool] = None):
        """``skinny``: decode projections on the skinny MFMA GEMM with fused epilogues (when the shapes allow);
        ``partials``: 2 = every projection leaves split-K slabs summed by its consumer (measured fastest,
        profiles/r2_decode_partials_ab.txt), 1 = the residual projections only, 0 = in-GEMM split-K hand-off;
        ``fused_sampler``: the one-kernel top-k / top-p / Gumbel sampler (K18); ``ln_tail`` (None: env
        DALLE_AMD_DECODE_LN_TAIL, default off): the out-proj / FF-out slabs and the next LayerNorm + shift in ONE
        launch (skinny EPI 5: the projection's last workgroups finish the rows) instead of the projection
        plus a decode_ln_shift launch -- 5 instead of 7 launches per layer, but measured slower
        (profiles/r6_decode_ln_tail.txt: 14.2 vs 16.8 images/s at batch 64; the in-launch hand-off's
        write-through, ticket, poll and read-back round trips cost more than the kernel boundary they remove).
        The non-default forms are kept for the numerics A/B in tests/test_generation_gpu.py."""
        self.model = model
        cfg = self.cfg = model.cfg
        self.B = batch_size
        self.device = device or next(model.parameters()).device
        dev = self.device
        if use_hip is None:
            from ..ops.ext import hip_available
            use_hip = dev.type == "cuda" and hip_available()
        self.use_hip = use_hip
        self.T, self.S, self.n = cfg.text_len, cfg.image_fmap_size, cfg.seq_len
        self.H, self.Dh, self.d = cfg.heads, cfg.dim_head, cfg.dim
        self.Vt = cfg.total_text_tokens
        self.cdt = torch.bfloat16 if use_hip else torch.float32
        tr = model.transformer
        self.pairs = tr.layers.pairs()
        self.geom = tr.geom
        L, B = len(self.pairs), batch_size
        self.kc = [torch.zeros(B * self.H, self.n, self.Dh, dtype=self.cdt, device=dev) for _ in range(L)]
        self.vc = [torch.zeros_like(k) for k in self.kc]
        self.hist = [[torch.zeros(B, self.n, self.d, dtype=self.cdt, device=dev) for _ in range(2)] for _ in range(L)]
        self.cos, self.sin = rotary_tables(self.T, self.S, self.Dh, device=dev)
        self.pos = torch.zeros((), dtype=torch.int32, device=dev)
        # 1 while every row carries the same caption (set per generate call, on device: a captured graph serves both
        # cases): the decode attention then reads the text positions' K / V from row 0's cache for all rows
        self.text_shared = torch.zeros(1, dtype=torch.int32, device=dev)
        self.share_text = True
        self.tok = torch.zeros(B, dtype=torch.long, device=dev)
        self.hbuf = torch.zeros(B, self.d, dtype=self.cdt, device=dev)
        self.qbuf = torch.zeros(B, self.H, self.Dh, dtype=self.cdt, device=dev)
        self.obuf = torch.zeros(B, self.H * self.Dh, dtype=self.cdt, device=dev)
        self.codes = torch.zeros(B, cfg.image_seq_len, dtype=torch.long, device=dev)
        self.temperature, self.top_k, self.top_p = 1.0, 0, 1.0
        # fused HIP sampler (K18); its Gumbel noise is a counter hash of (seed, position, row, token)
        self.fused_sampler = use_hip and fused_sampler
        self.seed = torch.zeros((), dtype=torch.int64, device=dev)
        self.graph = None
        self._pf_graphs = {}  # captured caption prefills, by (rows, input buffer)
        self._pf_masks = {}   # contiguous (P, P) caption blocks of the layer patterns
        self._static_logits = None
        self._w = {}
        # decode-step projections through the skinny MFMA GEMM (csrc/kernels/skinny.hip) with the
        # rotary / GEGLU / LayerScale-residual epilogues fused: M = batch <= 64 rows
        self.skinny = (use_hip and skinny and batch_size <= 64 and self.d % 128 == 0 and (cfg.ff_mult * self.d) % 128 == 0)
        self.sk_cnt = torch.zeros(8192, dtype=torch.int32, device=dev) if self.skinny else None
        # split-K partials: the projections leave fp32 slabs summed by their consumer, so those GEMMs
        # split K over 4-8x the workgroups with no cross-workgroup hand-off. 2 (default): out-proj /
        # FF-out slabs summed by the next LayerNorm, QKV slabs by the attention prologue (under the KV
        # stream); 1: residual projections only; 0: in-GEMM split-K hand-off
        # (profiles/r2_decode_partials_ab.txt: 4.02 -> 3.70-3.73 ms per image-position step)
        mode = int(partials) if self.skinny else 0
        self.partials = mode in (1, 2)
        self.qkv_partials = mode == 2
        # pending residual update of a stream, not yet applied: ("part", stream, slabs, bias, LayerScale) -- slabs
        # already computed -- or ("gemm", stream, X, W, bias, LayerScale) -- the projection itself deferred, so
        # that it runs as one launch with the LayerNorm that reads the stream (skinny_partials_ln_)
        self._pending = None
        if ln_tail is None:
            ln_tail = os.environ.get("DALLE_AMD_DECODE_LN_TAIL", "0") == "1"
        self.ln_tail = False
        if self.partials and ln_tail:
            from ..ops.hip_ops import C
            ok = C().skinny_partials_ln_ok
            self.ln_tail = ok(B, self.d, self.H * self.Dh) and ok(B, self.d, cfg.ff_mult * self.d)
        # one ticket word per fused launch site of a step (2 per layer), zeroed per generate call; error word
        self.ln_cnt = torch.zeros(2 * L + 2, dtype=torch.int32, device=dev) if self.ln_tail else None
        self.ln_err = torch.zeros(1, dtype=torch.int32, device=dev) if self.ln_tail else None
        self._site = 0

    # -- weights (one bf16 cast per generate call) --------------------------------------------------
    def _wt(self, p):
        ent = self._w.get(id(p))
        if ent is None:
            ent = (p, p.detach().to(self.cdt))
            self._w[id(p)] = ent
        return ent[1]

    _refresh_weights = True

    def reset(self):
        """Zero position/caches and refresh the compute-dtype weight copies IN PLACE (a captured graph
        keeps pointing at the same buffers, so weight updates between calls are still seen)."""
        self.pos.zero_()
        if self._refresh_weights:
            for p, w in self._w.values():
                w.copy_(p.detach().reshape(w.shape))
        for k in self.kc + self.vc:
            k.zero_()
        if self.ln_cnt is not None:
            self.ln_cnt.zero_()
            self.ln_err.zero_()

    # -- branch steps -------------------------------------------------------------------------------
    def _flush_pending(self):
        if self._pending is not None:
            from ..ops.hip_ops import C
            kind, x, *rest = self._pending
            self._pending = None
            if kind == "gemm":
                X, W, bias, scale = rest
                C().residual_from_partials_(x, C().skinny_partials(X, W), bias, scale)
            else:
                part, bias, scale = rest
                C().residual_from_partials_(x, part, bias, scale)

    def _ln_shift(self, ls, hist, x):
        pre = ls.fn
        if self.use_hip:
            from ..ops.hip_ops import C
            pend = self._pending
            if pend is not None and pend[1] is not x:
                self._flush_pending()
                pend = None
            self._pending = None
            if pend is not None and pend[0] == "gemm":
                _, _, X, W, pbias, pscale = pend
                site = self._site
                self._site += 1
                C().skinny_partials_ln_(X, W, pbias, pscale, x, pre.norm.weight.detach(), pre.norm.bias.detach(), hist,
                                        self.hbuf, self.pos, self.T, self.S, bool(pre.fn.enabled),
                                        self.ln_cnt[site:site + 1], self.ln_err)
                return self.hbuf
            part, pbias, pscale = (pend[2], pend[3], pend[4]) if pend is not None else (None, None, None)
            C().decode_ln_shift_(x, pre.norm.weight.detach(), pre.norm.bias.detach(), hist, self.hbuf, self.pos,
                                 self.T, self.S, bool(pre.fn.enabled), part, pbias, pscale)
            return self.hbuf
        y = F.layer_norm(x, (self.d,), pre.norm.weight, pre.norm.bias)
        p = int(self.pos)
        hist[:, p] = y
        if not pre.fn.enabled:
            return y
        out = y.clone()
        q, h2 = self.d // 4, self.d // 2
        if p < self.T:
            out[:, :h2] = hist[:, p - 1, :h2] if p >= 1 else 0.0
        else:
            k = p - self.T
            out[:, :q] = hist[:, p - self.S, :q] if k >= self.S else 0.0
            out[:, q:h2] = hist[:, p - 1, q:h2] if k % self.S else 0.0
        return out

    def _attn_res(self, li, ls, x_in, x_res):
        """x_res += LayerScale * Attention(LN-shift(x_in)); one skinny GEMM each for QKV (+rotary into
        the KV cache) and the output projection (+bias, LayerScale, residual) on the fused path."""
        if not self.skinny:
            return self._residual(x_res, self._attn(li, ls, x_in), ls)
        from ..ops.hip_ops import C
        attn = ls.fn.fn.fn
        h = self._ln_shift(ls, self.hist[li][0], x_in)
        if self.qkv_partials:
            part = C().skinny_partials(h, self._wt(attn.to_qkv.weight))
            C().decode_attn_part_(part, self.cos, self.sin, self.Dh ** -0.5, self.kc[li], self.vc[li], self.obuf, self.pos,
                                  self.T, self.S, self.H, self.geom.kernel_size, PATTERN_IDS[attn.attn_type], self.text_shared)
        else:
            C().skinny_qkv_rope_(h, self._wt(attn.to_qkv.weight), self.cos, self.sin, self.qbuf, self.kc[li], self.vc[li],
                                 self.pos, self.H, self.Dh ** -0.5, self.sk_cnt)
            C().decode_attn_(self.qbuf, self.kc[li], self.vc[li], self.obuf, self.pos, self.T, self.S, self.H,
                             self.geom.kernel_size, PATTERN_IDS[attn.attn_type], self.text_shared)
        if self.ln_tail:
            self._pending = ("gemm", x_res, self.obuf, self._wt(attn.to_out[0].weight), self._wt(attn.to_out[0].bias),
                             self._scale(ls))
            return x_res
        if self.partials:
            po = C().skinny_partials(self.obuf, self._wt(attn.to_out[0].weight))
            self._pending = ("part", x_res, po, self._wt(attn.to_out[0].bias), self._scale(ls))
            return x_res
        C().skinny_residual_(x_res, self.obuf, self._wt(attn.to_out[0].weight), self._wt(attn.to_out[0].bias),
                             self._scale(ls), self.sk_cnt)
        return x_res

    def _ff_res(self, li, ls, x_in, x_res):
        """x_res += LayerScale * FF(LN-shift(x_in)): FF1 with GEGLU and FF2 with the residual fused."""
        if not self.skinny:
            return self._residual(x_res, self._ff(li, ls, x_in), ls)
        from ..ops.hip_ops import C
        ff = ls.fn.fn.fn
        h = self._ln_shift(ls, self.hist[li][1], x_in)
        a = C().skinny_geglu(h, self._wt(ff.net[0].weight), self._wt(ff.net[0].bias), self.sk_cnt)
        if self.ln_tail:
            self._pending = ("gemm", x_res, a, self._wt(ff.net[3].weight), self._wt(ff.net[3].bias), self._scale(ls))
            return x_res
        if self.partials:
            self._pending = ("part", x_res, C().skinny_partials(a, self._wt(ff.net[3].weight)), self._wt(ff.net[3].bias),
                             self._scale(ls))
            return x_res
        C().skinny_residual_(x_res, a, self._wt(ff.net[3].weight), self._wt(ff.net[3].bias), self._scale(ls), self.sk_cnt)
        return x_res

    def _scale(self, ls):
        ent = self._w.get(("scale", id(ls.scale)))
        if ent is None:
            ent = (ls.scale, ls.scale.detach().reshape(-1).float().contiguous())
            self._w[("scale", id(ls.scale))] = ent
        return ent[1]

    def _attn(self, li, ls, x):
        attn = ls.fn.fn.fn
        h = self._ln_shift(ls, self.hist[li][0], x)
        qkv = F.linear(h, self._wt(attn.to_qkv.weight))
        if self.use_hip:
            from ..ops.hip_ops import C
            C().decode_rope_(qkv.contiguous(), self.cos, self.sin, self.qbuf, self.kc[li], self.vc[li], self.pos, self.H,
                             self.Dh ** -0.5)
            C().decode_attn_(self.qbuf, self.kc[li], self.vc[li], self.obuf, self.pos, self.T, self.S, self.H,
                             self.geom.kernel_size, PATTERN_IDS[attn.attn_type], self.text_shared)
            o = self.obuf
        else:
            o = self._attn_torch(li, attn, qkv)
        return F.linear(o, self._wt(attn.to_out[0].weight), self._wt(attn.to_out[0].bias))

    def _attn_torch(self, li, attn, qkv):
        from ..ops.reference import split_heads
        from .rotary import apply_rotary
        p = int(self.pos)
        B, H, Dh = self.B, self.H, self.Dh
        q, k, v = (t.view(B, H, 1, Dh) for t in qkv.chunk(3, dim=-1))
        c, s = self.cos[p:p + 1], self.sin[p:p + 1]
        q, k, v = (apply_rotary(t, c, s) for t in (q, k, v))
        kc = self.kc[li].view(B, H, self.n, Dh)
        vc = self.vc[li].view(B, H, self.n, Dh)
        kc[:, :, p] = k[:, :, 0]
        vc[:, :, p] = v[:, :, 0]
        mask = static_mask(self.geom, attn.attn_type, self.n, device=q.device)[p, : p + 1]
        sc = (q * Dh ** -0.5) @ kc[:, :, : p + 1].transpose(-1, -2)
        sc = sc.masked_fill(~mask, float("-inf"))
        o = torch.softmax(sc, -1) @ vc[:, :, : p + 1]
        return o.reshape(B, H * Dh)

    def _ff(self, li, ls, x):
        ff = ls.fn.fn.fn
        h = self._ln_shift(ls, self.hist[li][1], x)
        a = F.linear(h, self._wt(ff.net[0].weight), self._wt(ff.net[0].bias))
        if self.use_hip:
            from ..ops.hip_ops import C
            a = C().geglu_fwd(a.contiguous())
        else:
            a1, g = a.chunk(2, -1)
            a = a1 * F.gelu(g)
        return F.linear(a, self._wt(ff.net[3].weight), self._wt(ff.net[3].bias))

    def _residual(self, x, y, ls):
        """x += LayerScale * y (fp32 residual stream), one fused kernel on the HIP path."""
        if self.use_hip:
            from ..ops.hip_ops import C
            C().scale_residual_(x, y.contiguous(), ls.scale.detach().reshape(-1).contiguous())
            return x
        return x + y.float() * ls.scale.detach().view(1, -1)

    # -- one position through the whole network ------------------------------------------------------
    def _forward_position(self) -> torch.Tensor:
        W = self.model.to_logits[1].weight
        x = F.embedding(self.tok, W.detach()).float()
        self._pending = None
        self._site = 0
        if self.cfg.reversible:
            x1, x2 = x, x.clone()
            for li, (f, g) in enumerate(self.pairs):
                x1 = self._attn_res(li, f, x2, x1)
                x2 = self._ff_res(li, g, x1, x2)
            self._flush_pending()
            out = (x1 + x2) * 0.5
        else:
            for li, (f, g) in enumerate(self.pairs):
                x = self._attn_res(li, f, x, x)
                x = self._ff_res(li, g, x, x)
            self._flush_pending()
            out = x
        norm, head = self.model.to_logits[0], self.model.to_logits[1]
        h = F.layer_norm(out, (self.d,), norm.weight.detach(), norm.bias.detach())
        if self.skinny:
            from ..ops.hip_ops import C
            return C().skinny_linear(h.to(self.cdt), self._wt(head.weight)[self.Vt:], self._wt(head.bias)[self.Vt:], True,
                                     self.sk_cnt)
        return F.linear(h.to(self.cdt), self._wt(head.weight)[self.Vt:], self._wt(head.bias)[self.Vt:]).float()

    def _step(self):
        """Graph body for ANY position: run position ``pos``; choose the next input token on device --
        the next caption token while ``pos + 1 < T`` (prefill), else the sampled image token -- and
        record the sample as image code ``pos - T + 1`` (prefill writes are overwritten later)."""
        logits = self._forward_position()
        if self.fused_sampler and logits.dtype == torch.float32 and logits.shape[-1] <= 8192:
            # one HIP launch (csrc/kernels/sample.hip): filter + sample + codes / next-token bookkeeping
            from ..ops.hip_ops import C
            C().sample_step(logits, int(self.top_k or 0), float(1.0 if self.top_p is None else self.top_p),
                            float(self.temperature), self.seed, self.pos, self.text_bos, self.codes, self.tok, self.Vt)
            self.pos.add_(1)
            return logits
        logits = filter_logits(logits, self.top_k, self.top_p)
        nxt = gumbel_sample(logits, self.temperature)
        p = self.pos.long()
        idx = (p - (self.T - 1)).clamp(0, self.cfg.image_seq_len - 1).view(1, 1).expand(self.B, 1)
        self.codes.scatter_(1, idx, nxt.view(self.B, 1))
        nxt_text = self.text_bos.gather(1, (p + 1).clamp(max=self.T - 1).view(1, 1).expand(self.B, 1)).view(self.B)
        self.tok.copy_(torch.where(p + 1 < self.T, nxt_text, nxt + self.Vt))
        self.pos.add_(1)
        return logits

    _image_step = _step

    # -- public API ---------------------------------------------------------------------------------
    def _start(self, text_bos: torch.Tensor):
        self.reset()
        if not hasattr(self, "text_bos") or self.text_bos.shape != text_bos.shape:
            self.text_bos = torch.zeros_like(text_bos)
        self.text_bos.copy_(text_bos)
        self.tok.copy_(text_bos[:, 0])
        if self.share_text:
            self.text_shared.copy_((text_bos == text_bos[:1]).all().view(1))
        else:
            self.text_shared.zero_()

    @torch.no_grad()
    def prefill(self, text_bos: torch.Tensor):
        """Eagerly feed BOS + text positions 0..T-2 (position T-1 is the first sampling step)."""
        self._start(text_bos)
        for p in range(self.T - 1):
            self.tok.copy_(text_bos[:, p])
            self._forward_position()
            self.pos.add_(1)
        self.tok.copy_(text_bos[:, self.T - 1])

    # -- parallel prefill: the caption positions as ONE batched pass per layer -------------------------
    def _pf_ln_shift(self, ls, hist, x):
        """LN + cached token shift over all prefill positions at once: fills hist[:, :P] and returns the
        shifted rows (the text shift takes channels [0, d/2) from the previous position)."""
        pre = ls.fn
        P = x.shape[1]
        if self.use_hip and self.d in (256, 512, 1024, 2048):  # one kernel: LN, history rows, pushed shift
            from ..ops.hip_ops import C
            out = torch.empty(x.shape, dtype=self.cdt, device=x.device)
            C().prefill_ln_shift_(x, pre.norm.weight.detach(), pre.norm.bias.detach(), hist, out, bool(pre.fn.enabled),
                                  float(pre.norm.eps))
            return out
        y = F.layer_norm(x, (self.d,), pre.norm.weight.detach(), pre.norm.bias.detach(), pre.norm.eps).to(self.cdt)
        hist[:, :P] = y
        if not pre.fn.enabled:
            return y
        out = y.clone()
        h2 = self.d // 2
        out[:, 1:, :h2] = y[:, :-1, :h2]
        out[:, 0, :h2] = 0
        return out

    def _pf_attn(self, li, ls, x):
        attn = ls.fn.fn.fn
        B, P, H, Dh = x.shape[0], x.shape[1], self.H, self.Dh
        h = self._pf_ln_shift(ls, self.hist[li][0][:B], x)
        kc, vc = self.kc[li][: B * H], self.vc[li][: B * H]  # the first B rows' caches (all of them, or row 0)
        if self.use_hip:
            # the projections on the assembly GEMM where the rows tile (_pf_linear); one kernel rotates q / k / v and
            # writes k / v into the caches (q pre-scaled, bf16 as in the decode steps); scores in fp32, then one
            # masked-softmax kernel to bf16 probabilities. Returns the bf16 projection output (bias included).
            from ..ops.hip_ops import C
            qkv = self._pf_linear(h.view(B * P, self.d), attn.to_qkv.weight).view(B, P, -1)
            q = torch.empty(B * H, P, Dh, dtype=self.cdt, device=x.device)
            C().prefill_rope_(qkv, self.cos, self.sin, q, kc, vc, H, Dh ** -0.5)
            k, v = kc[:, :P], vc[:, :P]
            sc = torch.bmm(q, k.transpose(1, 2), out_dtype=torch.float32)
            mask = self._pf_mask(attn.attn_type, P, x.device)
            if P <= 512:  # the kernel keeps a row's scores in registers (8 per lane)
                pr = torch.empty(sc.shape, dtype=self.cdt, device=x.device)
                C().prefill_softmax_(sc, mask, pr)
            else:
                pr = torch.softmax(sc.masked_fill_(~mask, float("-inf")), -1).to(self.cdt)
            o = torch.bmm(pr, v)
            o = o.view(B, H, P, Dh).transpose(1, 2).reshape(B * P, H * Dh)
            return self._pf_linear(o, attn.to_out[0].weight, attn.to_out[0].bias).view(B, P, -1)
        qkv = F.linear(h, self._wt(attn.to_qkv.weight)).view(B, P, 3, H, Dh).permute(2, 0, 3, 1, 4).float()
        c, sn = self.cos[:P], self.sin[:P]
        q, k, v = (apply_rotary(t, c, sn) for t in qkv)
        kc.view(B, H, self.n, Dh)[:, :, :P] = k.to(self.cdt)
        vc.view(B, H, self.n, Dh)[:, :, :P] = v.to(self.cdt)
        # the cached (rounded) keys / values, as the decode steps will read them
        k, v = k.to(self.cdt).float(), v.to(self.cdt).float()
        sc = (q * Dh ** -0.5) @ k.transpose(-1, -2)
        mask = static_mask(self.geom, attn.attn_type, self.n, device=x.device)[:P, :P]
        o = torch.softmax(sc.masked_fill(~mask, float("-inf")), -1) @ v
        o = o.transpose(1, 2).reshape(B, P, H * Dh).to(self.cdt)
        return F.linear(o, self._wt(attn.to_out[0].weight), self._wt(attn.to_out[0].bias))

    def _pf_linear(self, x2, w, b=None):
        """x2 (M, K) bf16 . W^T (+ b) for the prefill: the assembly GEMM where the rows tile (its epilogue reads the
        fp32 bias parameter), else hipBLASLt -- with the engine's own bf16 copies either way, never the per-forward
        cast cache (a captured prefill must hold only buffers that outlive it)."""
        from ..ops.hip_ops import ASM_GEMM, C, _asm_ok
        wb = self._wt(w)
        if ASM_GEMM and _asm_ok(x2, wb) and (b is None or (b.dtype == torch.float32 and b.is_contiguous())):
            return C().asm_gemm(x2, wb, None if b is None else b.detach(), None)
        return F.linear(x2, wb, None if b is None else self._wt(b))

    def _pf_mask(self, attn_type: str, P: int, device):
        """The layer pattern's (P, P) caption block, contiguous (cached: the first, eager prefill fills it before
        the pass is captured)."""
        key = (attn_type, P)
        m = self._pf_masks.get(key)
        if m is None:
            m = static_mask(self.geom, attn_type, self.n, device=device)[:P, :P].contiguous()
            self._pf_masks[key] = m
        return m

    def _pf_ff(self, li, ls, x):
        ff = ls.fn.fn.fn
        B, P = x.shape[0], x.shape[1]
        h = self._pf_ln_shift(ls, self.hist[li][1][:B], x)
        if self.use_hip:
            from ..ops.hip_ops import C
            u = C().geglu_fwd(self._pf_linear(h.view(B * P, self.d), ff.net[0].weight, ff.net[0].bias))
            return self._pf_linear(u, ff.net[3].weight, ff.net[3].bias).view(B, P, -1)
        a = F.linear(h, self._wt(ff.net[0].weight), self._wt(ff.net[0].bias))
        val, gate = a.float().chunk(2, -1)
        u = (val * F.gelu(gate)).to(self.cdt)
        return F.linear(u, self._wt(ff.net[3].weight), self._wt(ff.net[3].bias))

    def _pf_add(self, x, ls, y):
        """x + LayerScale * y for a sublayer's projection output y: in place, one kernel, on MI355X."""
        if self.use_hip and self.d % 4 == 0:
            from ..ops.hip_ops import C
            C().prefill_residual_(x, y, self._scale(ls))
            return x
        return x + y.float() * self._scale(ls)

    def _pf_rows(self) -> int:
        """Rows the caption prefill runs for (after ``_start``): 1 when every row holds row 0's caption (a
        host read of the device flag: the one synchronisation of the prefill), else the batch."""
        one = self.use_hip and self.share_text and self.B > 1 and bool(self.text_shared.item())
        return 1 if one else self.B

    @torch.no_grad()
    def prefill_parallel(self, text_bos: torch.Tensor, rows: Optional[int] = None, started: bool = False):
        """Positions 0..T-2 (BOS + caption) as one batched pass per layer instead of T-1 decode steps:
        fills the KV caches and LN histories exactly where the steps would, then leaves the engine at
        position T-1 (the first sampling step) -- at batch 64 on the reference model this replaces
        ~0.9 s of sequential steps with a few ms.

        One caption repeated over the batch (the decode attention then reads the text keys / values from row
        0's cache, ``text_shared``): the pass runs for row 0 alone, and the other rows get only what the decode
        steps read of their own: the LN history at position T-2 (the shift of the first step, at T-1).
        ``rows`` / ``started``: given by a caller that already ran ``_start`` and ``_pf_rows`` (a split
        engine, which then launches the parts' passes on their streams with no host read in between)."""
        if not started:
            self._start(text_bos)
        P = self.T - 1
        if rows is None:
            rows = self._pf_rows()
        if P > 0:
            if self.use_hip:
                # the pass is ~25 launches per layer: captured once per (rows, input buffer) and replayed
                key = (rows, self.text_bos.data_ptr())
                graph = self._pf_graphs.get(key)
                if graph is None:
                    self._pf_body(rows, P)  # the result, and the libraries' warm-up for the capture
                    graph = torch.cuda.CUDAGraph()
                    with _CAPTURE_LOCK, torch.cuda.graph(graph, capture_error_mode="thread_local"):
                        self._pf_body(rows, P)
                    self._pf_graphs[key] = graph
                else:
                    graph.replay()
            else:
                self._pf_body(rows, P)
            self.pos.fill_(P)
        self.tok.copy_(text_bos[:, P])

    def _pf_body(self, rows: int, P: int):
        W = self.model.to_logits[1].weight.detach()
        x = F.embedding(self.text_bos[:rows, :P], W).float()
        if self.cfg.reversible:
            x1, x2 = x, x.clone()
            for li, (f, g) in enumerate(self.pairs):
                x1 = self._pf_add(x1, f, self._pf_attn(li, f, x2))
                x2 = self._pf_add(x2, g, self._pf_ff(li, g, x1))
        else:
            for li, (f, g) in enumerate(self.pairs):
                x = self._pf_add(x, f, self._pf_attn(li, f, x))
                x = self._pf_add(x, g, self._pf_ff(li, g, x))
        if rows < self.B:  # the other rows' own reads: the LN history the first decode step shifts in
            for hs in self.hist:
                for hb in hs:
                    hb[rows:, P - 1].copy_(hb[0, P - 1].expand(self.B - rows, -1))

    @torch.no_grad()
    def generate(self, text_bos: torch.Tensor, temperature: float = 1.0, top_k: int = 0, top_p: float = 1.0,
                 use_graph: Optional[bool] = None, seed: Optional[int] = None, parallel_prefill: Optional[bool] = None) -> torch.Tensor:
        """The caption prefill (one batched pass per layer, ``parallel_prefill``, default on; else T-1
        decode steps) then the 1024 sampled image tokens through one step function; on MI355X that step
        is a single hipGraph replayed per position. ``seed`` fixes the fused sampler's noise (default:
        drawn from torch's global generator)."""
        self.temperature, self.top_k, self.top_p = temperature, top_k, top_p
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.seed.fill_(int(seed))
        use_graph = self.use_hip if use_graph is None else use_graph
        if parallel_prefill is None:
            parallel_prefill = True
        self._start(text_bos)
        if use_graph:
            self._capture()
        steps = self.n
        if parallel_prefill:
            self.prefill_parallel(text_bos)
            steps = self.n - (self.T - 1)
        else:
            self._start(text_bos)
        for _ in range(steps):
            if use_graph:
                self.graph.replay()
            else:
                self._step()
        return self.codes.clone()

    def _capture(self):
        """Capture one image step into a hipGraph (warm-up on a side stream as torch requires)."""
        if self.graph is not None and self._graph_cfg == (self.temperature, self.top_k, self.top_p):
            return
        # warm-up on a side stream (allocator / library handles), then capture; the caller resets the
        # state (pos, tokens, caches) afterwards, so the warm-up steps leave no trace
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._step()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with _CAPTURE_LOCK, torch.cuda.graph(g, capture_error_mode="thread_local"):
            self._static_logits = self._step()
        self.graph = g
        self._graph_cfg = (self.temperature, self.top_k, self.top_p)

    @torch.no_grad()
    def teacher_forced_logits(self, text_bos: torch.Tensor, image: torch.Tensor) -> torch.Tensor:
        """Image-vocab logits at every position >= T-1 when feeding the given image codes (tests)."""
        self.prefill(text_bos)
        outs = []
        for i in range(self.cfg.image_seq_len):
            outs.append(self._forward_position())
            if i + 1 < self.cfg.image_seq_len:
                self.tok.copy_(image[:, i] + self.Vt)
                self.pos.add_(1)
        return torch.stack(outs, dim=1)


class _PartGraphs:
    """One image-position step of every part: each part's own captured graph replayed on the part's stream
    (the ``graph`` of a :class:`SplitDecodeEngine` in per-part mode)."""

    def __init__(self, eng):
        self.eng = eng

    def replay(self):
        self.eng.replay_steps(1)


class SplitDecodeEngine:
    """The batch split into ``parts`` independent :class:`DecodeEngine` s whose steps run concurrently
    on separate HIP streams. At batch 64 a decode step is a chain of short kernels whose time is mostly
    fixed latency (a skinny GEMM takes 8-10 us whether it streams 2 or 16 MB of weights), so two
    half-batch chains interleaved on the GPU overlap one chain's latency with the other's work. The
    parts share the bf16 weight copies; each has its own KV caches, LN histories, device position and
    sampler seed (``seed + part``), so the parts never touch the same buffer.

    ``graphs`` (``DALLE_AMD_DECODE_GRAPHS``): "per-part" (default) captures each part's step as its own
    LINEAR graph, replayed on the part's stream with no per-step join -- the HIP runtime launches a linear
    graph from pre-built packets, 0.17 ms of host time per step for both parts. "joint": one graph with the
    parts as parallel branches joined at the end of every step -- the runtime launches a multi-branch graph
    node by node, ~2.5 ms of host time per ~3 ms step, so the host barely stays ahead and its jitter reaches
    the GPU (profiles/r6_decode_replay_host.txt: 3.00-3.02 vs 3.05-3.11 ms per step)."""

    def __init__(self, model, batch_size: int, device=None, parts: int = 2, graphs: Optional[str] = None):
        if batch_size % parts:
            raise ValueError(f"batch {batch_size} is not divisible into {parts} parts")
        self.model, self.B, self.nparts = model, batch_size, parts
        self.parts = [DecodeEngine(model, batch_size // parts, device=device) for _ in range(parts)]
        for p in self.parts[1:]:
            p._w = self.parts[0]._w  # one bf16 copy of every weight, refreshed by part 0 only
            p._refresh_weights = False
        self.device = self.parts[0].device
        self.use_hip = self.parts[0].use_hip
        if graphs is None:
            graphs = os.environ.get("DALLE_AMD_DECODE_GRAPHS", "per-part")
        if graphs not in ("per-part", "joint"):
            raise ValueError(f"DALLE_AMD_DECODE_GRAPHS={graphs!r}: expected per-part or joint")
        self.graph_mode = graphs
        self.graph = None
        self._graph_cfg = None
        self._part_streams = None

    @property
    def codes(self) -> torch.Tensor:
        return torch.cat([p.codes for p in self.parts])

    def _start_all(self, text_bos: torch.Tensor):
        b = self.B // self.nparts
        for i, p in enumerate(self.parts):
            p._start(text_bos[i * b:(i + 1) * b])

    _start = _start_all

    def _step(self):
        for p in self.parts:
            p._step()

    _image_step = _step

    @torch.no_grad()
    def prefill(self, text_bos: torch.Tensor):
        b = self.B // self.nparts
        for i, p in enumerate(self.parts):
            p.prefill(text_bos[i * b:(i + 1) * b])

    @torch.no_grad()
    def prefill_parallel(self, text_bos: torch.Tensor):
        """Every part's caption prefill, the parts' passes concurrently on the part streams (with distinct
        captions each pass is ~0.7 ms of mid-size GEMMs per layer for 32 rows: run one after the other
        they took 93 ms per generate call). The shared-caption flags are read on the host first, so no
        synchronisation falls between the launches."""
        b = self.B // self.nparts
        slices = [text_bos[i * b:(i + 1) * b] for i in range(self.nparts)]
        for p, t in zip(self.parts, slices):
            p._start(t)
        rows = [p._pf_rows() for p in self.parts]
        if not self.use_hip:
            for p, t, r in zip(self.parts, slices, rows):
                p.prefill_parallel(t, rows=r, started=True)
            return
        if self._part_streams is None:
            self._part_streams = [torch.cuda.Stream() for _ in self.parts]
        main = torch.cuda.current_stream()
        for st in self._part_streams:
            st.wait_stream(main)
        for p, t, r, st in zip(self.parts, slices, rows, self._part_streams):
            with torch.cuda.stream(st):
                p.prefill_parallel(t, rows=r, started=True)
        for st in self._part_streams:
            main.wait_stream(st)

    def _capture(self):
        cfg = (self.parts[0].temperature, self.parts[0].top_k, self.parts[0].top_p)
        if self.graph is not None and self._graph_cfg == cfg:
            return
        if self.graph_mode == "per-part":
            for p in self.parts:
                p._capture()  # a linear graph of the part's own step (its warm-up steps are reset by the prefill)
            if self._part_streams is None:
                self._part_streams = [torch.cuda.Stream() for _ in self.parts]
            self.graph = _PartGraphs(self)
            self._graph_cfg = cfg
            return
        main = torch.cuda.current_stream()
        streams = [torch.cuda.Stream() for _ in self.parts[1:]]
        warm = torch.cuda.Stream()
        warm.wait_stream(main)
        with torch.cuda.stream(warm):
            for _ in range(2):
                for p in self.parts:
                    p._step()
        main.wait_stream(warm)
        g = torch.cuda.CUDAGraph()
        with _CAPTURE_LOCK, torch.cuda.graph(g, capture_error_mode="thread_local"):
            cap = torch.cuda.current_stream()
            for s in streams:
                s.wait_stream(cap)
            self.parts[0]._step()
            for p, s in zip(self.parts[1:], streams):
                with torch.cuda.stream(s):
                    p._step()
            for s in streams:
                cap.wait_stream(s)
        self.graph = g
        self._streams = streams
        self._graph_cfg = cfg

    @torch.no_grad()
    def generate(self, text_bos: torch.Tensor, temperature: float = 1.0, top_k: int = 0, top_p: float = 1.0,
                 use_graph: Optional[bool] = None, seed: Optional[int] = None) -> torch.Tensor:
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        for i, p in enumerate(self.parts):
            p.temperature, p.top_k, p.top_p = temperature, top_k, top_p
            p.seed.fill_(int(seed) + i)
        use_graph = self.use_hip if use_graph is None else use_graph
        n = self.parts[0].n
        self._start_all(text_bos)
        if use_graph:
            self._capture()
        self.prefill_parallel(text_bos)
        steps = n - (self.parts[0].T - 1)
        if use_graph:
            self.replay_steps(steps)
        else:
            for _ in range(steps):
                for p in self.parts:
                    p._step()
        return self.codes.clone()

    def replay_steps(self, k: int):
        """``k`` decode steps through the captured graph(s). Per-part: the part streams fork from the current
        stream, each replays its part's graph ``k`` times with no join in between, and the current stream
        joins them at the end (the codes are read there)."""
        if self.graph_mode == "joint":
            for _ in range(k):
                self.graph.replay()
            return
        main = torch.cuda.current_stream()
        for st in self._part_streams:
            st.wait_stream(main)
        for _ in range(k):
            for p, st in zip(self.parts, self._part_streams):
                with torch.cuda.stream(st):
                    p.graph.replay()
        for st in self._part_streams:
            main.wait_stream(st)


def decode_parts(batch_size: int, device, parts: Optional[int] = None) -> int:
    """How many concurrent batch-slice chains a decode engine uses: ``parts`` (else ``DALLE_AMD_DECODE_PARTS``),
    default 2 for batches of 32 and more (1 below); 4 chains measured 17.7 vs 20.1 images/s with per-part graphs
    (profiles/r6_decode_replay_host.txt). Reference model, batch 64, same box
    (profiles/r2_decode_split_parts.txt): 2 parts 3.53 ms per image-position step and 17.0 images/s vs
    3.74 ms / 16.0 for one chain; 4 parts 4.0-6.1 ms. With the decode kernels at a few us each, two
    half-batch chains overlap one chain's latency-bound kernels with the other's (it measured +1 % when
    the skinny GEMMs still carried their split-K hand-off)."""
    if parts is None and os.environ.get("DALLE_AMD_DECODE_PARTS"):
        parts = int(os.environ["DALLE_AMD_DECODE_PARTS"])
    n = max(1, int(parts if parts is not None else (2 if batch_size >= 32 else 1)))
    return n if batch_size % n == 0 else 1


def make_decode_engine(model, batch_size: int, device=None):
    device = device or next(model.parameters()).device
    parts = decode_parts(batch_size, device)
    if parts > 1:
        eng = SplitDecodeEngine(model, batch_size, device=device, parts=parts)
        if eng.use_hip:
            return eng
    return DecodeEngine(model, batch_size, device=device)
