"""HIP execution path: autograd Functions over the ``dalle_amd._C`` kernels + hipBLASLt GEMMs.

Numerics: fp32 residual stream and fp32 master weights; bf16 GEMM operands / activations with
fp32 accumulation; weight gradients are produced directly in fp32 by the GEMM
(``torch.mm(..., out_dtype=float32)`` -> hipBLASLt bf16-in / fp32-out), so gradients of the shared
blocks (summed over every layer that reuses them) never round through bf16.
"""
from __future__ import annotations

import os
import weakref
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from .ext import load_extension
from ..models.patterns import PATTERN_IDS, AttnGeometry
from ..models.rotary import rotary_tables

_C = None

# how often each fused path ran (tests assert that the fast paths -- not a fallback -- were exercised)
PATH_COUNTS: Dict[str, int] = {}


def _count(path: str):
    PATH_COUNTS[path] = PATH_COUNTS.get(path, 0) + 1


class _SyncedExtension:
    """``DALLE_AMD_DEBUG_SYNC=1``: every native op is followed by a device synchronisation,
    so an asynchronous fault or a race surfaces at the op that caused it, with its name."""

    def __init__(self, ext):
        self._ext = ext

    def __getattr__(self, name):
        fn = getattr(self._ext, name)

        def synced(*args, **kwargs):
            out = fn(*args, **kwargs)
            try:
                torch.cuda.synchronize()
            except RuntimeError as e:
                raise RuntimeError(f"dalle_amd._C.{name} failed on the device: {e}") from e
            return out
        return synced


def C():
    global _C
    if _C is None:
        ext = load_extension(required=True)
        _C = _SyncedExtension(ext) if os.environ.get("DALLE_AMD_DEBUG_SYNC") == "1" else ext
    return _C


# ---------------------------------------------------------------------------------------------
# bf16 weight cast cache (one cast per unique weight per forward; invalidated by begin_forward)
# ---------------------------------------------------------------------------------------------
_wcache: Dict[object, Tuple[object, tuple, torch.Tensor]] = {}
_epoch = 0


def begin_forward():
    global _epoch
    _epoch += 1
    _wcache.clear()


def _cached(key, w: torch.Tensor, make):
    """Per-weight cache entry. A hit needs the SAME live tensor (weak reference: a recycled id() and a
    recycled storage address of a new tensor never match a dead one's entry) at the same address, shape
    and version counter; begin_forward() clears everything per forward, which covers the optimizer's
    raw-pointer updates."""
    stamp = (w.data_ptr(), tuple(w.shape), w._version)
    hit = _wcache.get(key)
    if hit is not None and hit[0]() is w and hit[1] == stamp:
        return hit[2]
    val = make()
    _wcache[key] = (weakref.ref(w), stamp, val)
    return val


def bf16_weight(w: torch.Tensor) -> torch.Tensor:
    if w.dtype == torch.bfloat16:
        return w
    return _cached(id(w), w, lambda: w.detach().to(torch.bfloat16))


def bf16_weight_t(w: torch.Tensor) -> torch.Tensor:
    """Transposed (in, out) bf16 copy of a Linear weight, cached per forward like ``bf16_weight``: the
    B operand of an NT GEMM that multiplies by W instead of W^T (the fused FF dgrad)."""
    def make():
        if w.is_cuda and w.dtype == torch.float32 and w.dim() == 2 and w.is_contiguous():
            return C().transpose_bf16(w)  # one tiled pass instead of a cast + a strided copy
        return bf16_weight(w).t().contiguous()

    return _cached(("t", id(w)), w, make)


# Plain projections (no fused epilogue beyond a bias) run on the hand-scheduled assembly GEMM
# (csrc/asm/gen_gemm.py: hipBLASLt's own gfx950 structure -- 4 waves, 128x128 AGPR quadrants, LDS-DMA two
# K-steps ahead -- with every instruction placed by the generator) wherever the shape tiles; hipBLASLt
# otherwise. DALLE_AMD_ASM_GEMM=0 sends every plain product to hipBLASLt (A/B).
ASM_GEMM = os.environ.get("DALLE_AMD_ASM_GEMM", "1") != "0"


def _asm_ok(a: torch.Tensor, b: torch.Tensor) -> bool:
    return (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 2
            and a.stride(1) == 1 and b.stride(1) == 1 and a.shape[0] % 256 == 0 and b.shape[0] % 256 == 0
            and a.shape[1] % 128 == 0 and a.shape[1] >= 256 and a.shape[1] == b.shape[1])


def mm_nt(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """a (M, K) . b (N, K)^T (+ bias, the fp32 parameter): the assembly GEMM where the shape tiles, else
    hipBLASLt (with the bias rounded to bf16, the library's epilogue type)."""
    if ASM_GEMM and _asm_ok(a, b):
        _count("asm_gemm")
        bf = None if bias is None else bias.detach().float().contiguous()
        return C().asm_gemm(a, b, bf, None)
    if bias is not None:
        return torch.addmm(bf16_weight(bias), a, b.t())
    return torch.mm(a, b.t())


_perms: Dict[tuple, torch.Tensor] = {}


def ff_in_perm(F: int, device) -> torch.Tensor:
    """Row order of W1 (and b1) for the fused FF-in + GEGLU kernel: 4-row blocks [value j..j+3 | gate j..j+3],
    so each lane's 8 output columns are the values and gates of 4 j (csrc/asm/gen_gemm.py kernel_geglu)."""
    key = (F, str(device))
    p = _perms.get(key)
    if p is None:
        n = torch.arange(2 * F, device=device)
        p = 4 * (n >> 3) + (n & 3) + ((n >> 2) & 1) * F
        _perms[key] = p
    return p


def asm_fused_k(d: int) -> bool:
    """the fused assembly kernels (QKV + rotary, FF-in + GEGLU, FF-dgrad + GEGLU backward) take K = d_model a
    multiple of 128 and >= 1024: their successor tile's first 14 K-steps are unrolled (gen_gemm.FUSED_UNROLL),
    the rest runs in the ordinary K-loop -- d = 1024 (bench24 / reference) and d = 2048 (the ~1.3B preset)"""
    return d >= 1024 and d % 128 == 0


def _ff_in_geglu_ok(h2: torch.Tensor, w1: torch.Tensor) -> bool:
    return (ASM_GEMM and h2.is_cuda and h2.dtype == torch.bfloat16 and h2.dim() == 2 and h2.stride(1) == 1
            and asm_fused_k(h2.shape[1]) and h2.shape[0] % 256 == 0 and w1.shape[0] % 256 == 0
            and w1.shape[1] == h2.shape[1])


def ff_in_geglu(h2: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor):
    """(a, u) = (h2 W1^T + b1, GEGLU(a)) in one assembly kernel (u computed from the stored bf16 a, as the
    separate geglu kernel would); W1 / b1 are permuted once per forward (cached like the bf16 casts)."""
    F = w1.shape[0] // 2
    perm = ff_in_perm(F, w1.device)
    w1p = _cached(("ffw", id(w1)), w1, lambda: bf16_weight(w1).index_select(0, perm).contiguous())
    b1p = _cached(("ffb", id(b1)), b1, lambda: b1.detach().float().index_select(0, perm).contiguous())
    _count("asm_ff_in_geglu")
    return C().asm_ff_in_geglu(h2, w1p, b1p)


def input_grad(g: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """dX = g W for a Linear weight W (out, in), computed as g . (W^T)^T from the cached transposed bf16
    copy: the NT form of the product (hipBLASLt also runs it 12-20 % faster than the NN form at every
    training input-gradient shape, profiles/r2_gemm_layouts.jsonl)."""
    return mm_nt(g, bf16_weight_t(w))


_tables: Dict[tuple, tuple] = {}


def _rope_tables(geom: AttnGeometry, dim_head: int, device):
    key = (geom.text_len, geom.image_size, dim_head, str(device))
    t = _tables.get(key)
    if t is None:
        t = rotary_tables(geom.text_len, geom.image_size, dim_head, device=device)
        _tables[key] = t
    return t


_cs_tables: Dict[tuple, torch.Tensor] = {}
_rot_freq_cache: Dict[str, tuple] = {}


def _rot_freqs(device) -> tuple:
    """(rotf, n_lang, n_pix, image_text_pos, text_axial_pos) of the 64-dim heads on ``device`` (cached): the fused
    attention backward computes the rotary angles in-kernel from these (rotary.rotary_freq_split)."""
    key = str(device)
    t = _rot_freq_cache.get(key)
    if t is None:
        from ..models.rotary import rotary_freq_split

        t = rotary_freq_split(64, device)
        _rot_freq_cache[key] = t
    return t


def rope_cs_table(geom: AttnGeometry, dim_head: int, device) -> torch.Tensor:
    """(n + 1, dim_head / 2, 2) fp32 (cos, sin) per rotary pair -- the packed form of the rotary tables
    read by the persistent QKV GEMM's epilogue (pairs share their cos; the rotate_half sign is applied
    in the kernel)."""
    key = (geom.text_len, geom.image_size, dim_head, str(device))
    t = _cs_tables.get(key)
    if t is None:
        cos, sin = _rope_tables(geom, dim_head, device)
        t = torch.stack([cos[:, 0::2], sin[:, 1::2]], dim=-1).contiguous()
        _cs_tables[key] = t
    return t


def _cs3_from_tables(cos: torch.Tensor, sin: torch.Tensor, qscale: float) -> torch.Tensor:
    """(3, n + 1, 32, 2) (cos, sin) per rotary pair for q (scaled by ``qscale``), k and v (all three are rotated,
    as rope_fwd does): the table of the assembly QKV + rotary kernel (cached per table)."""
    key = ("cs3", cos.data_ptr(), tuple(cos.shape), str(cos.device), qscale)
    t = _cs_tables.get(key)
    if t is None:
        cs = _cs_from_tables(cos, sin)
        t = torch.stack([cs * qscale, cs, cs]).contiguous()
        _cs_tables[key] = t
    return t


def _cs_from_tables(cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """rope_cs_table's packing from the (cos, sin) tables themselves (cached per table)."""
    key = ("tab", cos.data_ptr(), tuple(cos.shape), str(cos.device))
    t = _cs_tables.get(key)
    if t is None:
        t = torch.stack([cos[:, 0::2], sin[:, 1::2]], dim=-1).contiguous()
        _cs_tables[key] = t
    return t


# ---------------------------------------------------------------------------------------------
# Linear: bf16 GEMM forward, fp32 weight grads accumulated straight into the fp32 grad buffer
# ---------------------------------------------------------------------------------------------
FUSE_WGRAD = True


def wgrad_splits(M: int, N: int, K: int) -> int:
    """Split-K factor for a weight-grad GEMM (N x K output, reduction over M tokens). Measured on
    MI355X at M = 61440 (profiles/r1_gemm_wgrad_m61440.jsonl, TF at 1/2/4/8 splits): 1024x1024
    405/533/687/834, 3072x1024 718/929/1009/984, 1024x4096 965/1007/1083/1032, 8192x1024
    1077/1125/1114/1053; at M = 81920 (micro-batch 64, profiles/r3_wgrad_splits_m81920.txt) the same
    choices win except 1024x1024, where 16 splits beat 8 (936 vs 904 TF)."""
    nk = N * K
    s = (16 if M >= 81920 else 8) if nk <= 1536 * 1024 else (4 if nk <= 4608 * 1024 else 2)
    while s > 1 and (M % s or M // s < 1024):
        s //= 2
    return s


# the QKV projection runs on the hand-written GEMM with the rotary in its register epilogue, writing the attention
# storage layout directly (csrc/kernels/gemm_pt.hip: 427 us vs 473 us for hipBLASLt + a rotary pass at the
# bench24 B48 shape, profiles/r3_gemm_pt_vs_hipblaslt_8ph.jsonl); the rotary backward runs in the attention-
# backward epilogues and the GEGLU backward in the FF-out dgrad GEMM's epilogue (csrc/kernels/gemm.hip EPI 2).


# weight-grad inputs kept token-contiguous: the LN outputs feeding the QKV and FF-in GEMMs are saved as
# X^T (one bf16 transpose kernel, ~60 us per 168 MB) instead of X, and dW = g^T X runs on hipBLASLt with
# a token-contiguous B operand: 3072x1024 1128 vs 847 TF/s, 8192x1024 1334 vs 1130 at M = 81920
# (profiles/r3s5_wgrad_nt_vs_tn_m81920.txt).
WGRAD_XT = not ASM_GEMM   # the assembly TN weight-grad kernel reads token-major inputs directly


class XT:
    """A saved GEMM input held transposed: ``t`` is X^T (K x M, contiguous bf16) of the logical X (M x K)."""

    __slots__ = ("t",)

    def __init__(self, t: torch.Tensor):
        self.t = t

    @property
    def shape(self):
        return (self.t.shape[1], self.t.shape[0])


# the FF-out weight grad also takes its output grad token-contiguous (dy^T: one transient transpose, 54-62 us
# per 168 MB; the 1024x4096 product runs at 1265 vs 1106 TF/s in isolation): small but consistent in the full
# step -- micro-batch 64 229.50 / 229.41 vs 229.54 / 229.63 ms, micro-batch 128 459.41 / 458.95 vs 460.09 /
# 461.66 ms (same box each, profiles/r3s5_wgrad_xt_ab.txt)
WGRAD_GT = not ASM_GEMM


def saved_gemm_input(x2: torch.Tensor, enabled: Optional[bool] = None):
    """``x2`` as the weight-grad GEMM will want it in the backward: ``XT`` when WGRAD_XT applies."""
    if ((WGRAD_XT if enabled is None else enabled) and x2.is_cuda and x2.dtype == torch.bfloat16 and x2.dim() == 2 and x2.is_contiguous()
            and x2.shape[0] % 64 == 0 and x2.shape[1] % 64 == 0):
        _count("wgrad_xt")
        return XT(C().transpose_act_bf16(x2))
    return x2


def wgrad_t_splits(M: int, N: int, K: int, form: str) -> int:
    """Split-K factor of the token-contiguous weight-grad forms, measured at M = 81920 (TF/s at 2/4/8/16
    splits, profiles/r3s5_wgrad_xt_ab.txt). ``xt`` (X^T given): 3072x1024 884/1050/1088/1128, 1024x1024
    515/670/1000/1112, 8192x1024 1334/1309/1294/1222, 1024x4096 1208/1241/1209/1142. ``gt`` (G^T given):
    3072x1024 884/1083/1108/1192, 1024x1024 535/664/942/1108, 8192x1024 1316/1283/1246/1195, 1024x4096
    1232/1238/1265/1148. ``nt`` (both): 3072x1024 1140/1255/1239/1237, 8192x1024 1406/1416/1377/1288,
    1024x4096 1285/1348/1365/1281."""
    nk = N * K
    if form == "gt":
        s = 16 if nk <= 3072 * 1024 else (8 if nk <= 4608 * 1024 else 2)
    elif form == "nt":
        s = 16 if nk <= 1536 * 1024 else (8 if nk <= 4608 * 1024 else 4)
    else:
        s = 16 if nk <= 3072 * 1024 else (4 if nk <= 4608 * 1024 else 2)
    while s > 1 and (M % s or M // s < 1024):
        s //= 2
    return s


def _weight_grad_t(gw, fused: bool, g2, x2):
    """dW = g^T x with G and/or X given token-contiguous (XT): split-K batched hipBLASLt GEMM whose
    operands are strided views of the transposed copies (no gather), fp32 partials + the fold kernel."""
    gt = g2.t if isinstance(g2, XT) else None
    xt = x2.t if isinstance(x2, XT) else None
    M, N = g2.shape
    K = x2.shape[1]
    form = "nt" if (gt is not None and xt is not None) else ("gt" if gt is not None else "xt")
    s = wgrad_t_splits(M, N, K, form)
    ms = M // s
    a = gt.view(N, s, ms).transpose(0, 1) if gt is not None else g2.view(s, ms, N).transpose(1, 2)
    b = xt.view(K, s, ms).transpose(0, 1).transpose(1, 2) if xt is not None else x2.view(s, ms, K)
    if s > 1:
        out = gw if fused else torch.empty(N, K, dtype=torch.float32, device=a.device)
        part = torch.bmm(a, b, out_dtype=torch.float32)
        C().splitk_accum_(out, part, fused)
        return None if fused else out
    if fused:
        torch.addmm(gw, a[0], b[0], out_dtype=torch.float32, out=gw)
        return None
    return torch.mm(a[0], b[0], out_dtype=torch.float32)


def asm_wgrad_splits(M: int, N: int, K: int) -> int:
    """Split count of the assembly TN weight-grad kernel for an (N x K) weight over M tokens, or 0 when the
    shape does not tile. Cost model: the main loop takes (whole waves of the 256 CUs the (tile, split) units
    occupy) x (work per unit), at ~1.45 PF/s; every split adds an fp32 partial slab that is written and read
    back by the fold (8 B per weight element, ~5 TB/s). Checked with sustained A/B runs at M = 163840
    (profiles/r5_ab_sustained.txt): 3072x1024 s5 732 us vs s16 768 (the old whole-wave rule picked 16),
    1024x1024 s16 264 vs s10 317, 1024x4096 s4 957 vs s5 1264; 8192x1024 stays at s2."""
    if N % 256 or K % 256:
        return 0
    tiles = (N // 256) * (K // 256)
    main = 2.0 * M * N * K / 1.45e15
    best = None
    for s in (1, 2, 4, 5, 8, 10, 16, 20, 32):
        if M % (128 * s) or M // s < 256:
            continue
        units = tiles * s
        waves = -(-units // 256)
        cost = main * waves * 256 / units + s * N * K * 8 / 5e12
        if best is None or cost < best[0]:
            best = (cost, s)
    return best[1] if best else 0


def _asm_wgrad_ok(g2, x2) -> bool:
    return (ASM_GEMM and isinstance(g2, torch.Tensor) and isinstance(x2, torch.Tensor) and g2.is_cuda
            and g2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 and g2.dim() == 2 and x2.dim() == 2
            and g2.stride(1) == 1 and x2.stride(1) == 1 and g2.shape[0] == x2.shape[0])


def weight_grad(w: torch.Tensor, g2: torch.Tensor, x2):
    """dW = g2^T x2 in fp32. When ``w.grad`` already exists (the flat grad arena), accumulate into it
    and return None: no temporary dW and no autograd add kernel, and the shared blocks' grads (one per
    reusing layer) sum in fp32. Small outputs run as a split-K batched GEMM (fp32 partials) + one
    deterministic fold kernel; large ones accumulate inside the GEMM (hipBLASLt beta = 1). ``x2`` and / or
    ``g2`` may be an ``XT`` (token-contiguous transposed copy, see saved_gemm_input)."""
    gw = w.grad
    fused = FUSE_WGRAD and gw is not None and gw.dtype == torch.float32 and gw.is_contiguous() and gw.shape == w.shape
    if isinstance(x2, XT) or isinstance(g2, XT):
        return _weight_grad_t(gw, fused, g2, x2)
    M, N, K = g2.shape[0], g2.shape[1], x2.shape[1]
    if _asm_wgrad_ok(g2, x2):
        s = asm_wgrad_splits(M, N, K)
        if s:
            _count("asm_wgrad")
            out = gw if fused else torch.empty(N, K, dtype=torch.float32, device=g2.device)
            C().asm_wgrad_(out, g2, x2, s, fused)
            return None if fused else out
    s = wgrad_splits(M, N, K)
    if s > 1:
        out = gw if fused else torch.empty(N, K, dtype=torch.float32, device=g2.device)
        part = torch.bmm(g2.view(s, M // s, N).transpose(1, 2), x2.view(s, M // s, K), out_dtype=torch.float32)
        C().splitk_accum_(out, part, fused)
        return None if fused else out
    if fused:
        torch.addmm(gw, g2.t(), x2, out_dtype=torch.float32, out=gw)
        return None
    return torch.mm(g2.t(), x2, out_dtype=torch.float32)


def grad_sink(p: torch.Tensor, needed: bool = True):
    """The fp32 ``.grad`` buffer (flattened view) a kernel may accumulate ``p``'s gradient into, or None
    (then the op returns the gradient to autograd as usual). Same contract as ``weight_grad``."""
    if not (FUSE_WGRAD and needed):
        return None
    g = p.grad
    if g is not None and g.dtype == torch.float32 and g.is_contiguous() and g.shape == p.shape:
        return g.view(-1)
    return None


def _bf16c(t):
    t = t if t.dtype == torch.bfloat16 else t.to(torch.bfloat16)
    return t.contiguous()


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        wb = bf16_weight(w)
        x2 = x.reshape(-1, x.shape[-1])
        if b is not None:
            y = torch.addmm(bf16_weight(b), x2, wb.t())
        else:
            y = torch.mm(x2, wb.t())
        ctx.save_for_backward(x2, wb)
        ctx.w = w
        ctx.has_bias = b is not None
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, wb = ctx.saved_tensors
        g2 = _bf16c(gy.reshape(-1, gy.shape[-1]))
        dx = input_grad(g2, ctx.w).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        dw = weight_grad(ctx.w, g2, x2) if ctx.needs_input_grad[1] else None
        db = torch.sum(g2, 0, dtype=torch.float32) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db


class _FF1GEGLU(torch.autograd.Function):
    """FF-in GEMM (+bias) -> GEGLU; backward = fused GEGLU-bwd + bias-grad kernel, then two GEMMs."""

    @staticmethod
    def forward(ctx, h, w, b):
        wb = bf16_weight(w)
        h2 = _bf16c(h.reshape(-1, h.shape[-1]))
        a = torch.addmm(bf16_weight(b), h2, wb.t())
        out = C().geglu_fwd(a)
        ctx.save_for_backward(h2, a, wb)
        ctx.w = w
        ctx.hshape = h.shape
        return out.view(*h.shape[:-1], out.shape[-1])

    @staticmethod
    def backward(ctx, gout):
        h2, a, wb = ctx.saved_tensors
        g = _bf16c(gout.reshape(a.shape[0], -1))
        da, db = C().geglu_bwd_bias(a, g)
        dh = input_grad(da, ctx.w).view(ctx.hshape)
        dw = weight_grad(ctx.w, da, h2)
        return dh, dw, db


class _ProjResidual(torch.autograd.Function):
    """out = x + scale * (o W^T + b): output GEMM with the LayerScale + residual epilogue (K8/K10).
    Backward: one kernel produces dy = bf16(scale*g), dscale = colsum(g*y) and colsum(g) (-> dbias)."""

    @staticmethod
    def forward(ctx, x, o, w, b, scale):
        wb = bf16_weight(w)
        o2 = _bf16c(o.reshape(-1, o.shape[-1]))
        y = torch.addmm(bf16_weight(b), o2, wb.t())
        s = scale.reshape(-1).contiguous()
        out = torch.empty_like(x)
        C().scale_residual_out(x.contiguous(), y, s, out)
        ctx.save_for_backward(o2, y, wb, s)
        ctx.w = w
        ctx.oshape, ctx.sshape = o.shape, scale.shape
        return out

    @staticmethod
    def backward(ctx, g):
        o2, y, wb, s = ctx.saved_tensors
        dy, dscale, gsum = C().scale_residual_bwd(g.contiguous(), y, s)
        dy = dy.view(-1, dy.shape[-1])
        do = input_grad(dy, ctx.w).view(ctx.oshape)
        dw = weight_grad(ctx.w, dy, o2)
        db = gsum * s
        return g, do, dw, db, dscale.view(ctx.sshape)


def ff_hidden(h, w1, b1):
    return _FF1GEGLU.apply(h, w1, b1)


def proj_residual(x, o, w, b, scale):
    return _ProjResidual.apply(x, o, w, b, scale)


def linear(x, w, b=None):
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    return _Linear.apply(x, w, b)


# ---------------------------------------------------------------------------------------------
# K1 + K2: token ids + gather from the tied fp32 table; backward = deterministic segmented row sums
# straight into the table's arena gradient (csrc/kernels/embed.hip)
# ---------------------------------------------------------------------------------------------
class _Embed(torch.autograd.Function):
    @staticmethod
    def forward(ctx, text, image, weight, pad_base: int, Vt: int):
        out, ids, bad = C().embed_fwd(text.contiguous(), image.contiguous(), weight.detach().contiguous(), int(pad_base),
                                      int(Vt))
        ctx.save_for_backward(ids)
        ctx.w = weight
        ctx.bad = bad  # device flag: an id outside the table was clamped (checked by tests / debug tools)
        _count("embed")
        return out

    @staticmethod
    def backward(ctx, g):
        (ids,) = ctx.saved_tensors
        w = ctx.w
        g2 = g.reshape(-1, g.shape[-1]).float().contiguous()
        sorted_ids, order = torch.sort(ids, stable=True)
        n = ids.numel()
        pos = torch.arange(n, device=ids.device, dtype=torch.int64)
        start = torch.ones(n, dtype=torch.bool, device=ids.device)
        start[1:] = sorted_ids[1:] != sorted_ids[:-1]
        head = torch.cummax(torch.where(start, pos, torch.zeros_like(pos)), 0).values.to(torch.int32)
        sink = grad_sink(w, ctx.needs_input_grad[2])
        if sink is not None:
            C().embed_bwd_(g2, order.to(torch.int32), sorted_ids.contiguous(), head, sink.view(w.shape))
            return None, None, None, None, None
        dw = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
        C().embed_bwd_(g2, order.to(torch.int32), sorted_ids.contiguous(), head, dw)
        return None, None, dw, None, None


def embed_tokens(text, image, weight, pad_base: int, Vt: int):
    """fp32 tokens (B, n, d) of [BOS | text (0 -> unique pad id) | image codes + Vt][:-1] from ``weight``."""
    return _Embed.apply(text, image, weight, pad_base, Vt)


# ---------------------------------------------------------------------------------------------
# K3+K4: LayerNorm + token shift
# ---------------------------------------------------------------------------------------------
class _LNShift(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, T, S, shift):
        x = x.contiguous()
        y, mean, rstd = C().ln_shift_fwd(x, w.contiguous(), b.contiguous(), T, S, shift, 1e-5)
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.geo = (T, S, shift)
        ctx.params = (w, b)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, mean, rstd = ctx.saved_tensors
        T, S, shift = ctx.geo
        gy = gy.to(torch.bfloat16).contiguous()
        sk = _sinks(ctx.params, ctx.needs_input_grad[1:3])
        if sk is not None:
            dx, dw, db = C().ln_shift_bwd(x, w.contiguous(), gy, mean, rstd, T, S, shift, None, sk[0], sk[1])
        else:
            dx, dw, db = C().ln_shift_bwd(x, w.contiguous(), gy, mean, rstd, T, S, shift)
        return dx, dw, db, None, None, None


def layernorm_shift(x, weight, bias, text_len: int, image_size: int, shift: bool = True):
    if x.dtype != torch.float32:
        x = x.float()
    return _LNShift.apply(x, weight, bias, text_len, image_size, bool(shift))


# ---------------------------------------------------------------------------------------------
# K6 + K7: rotary + sparse attention core
# ---------------------------------------------------------------------------------------------
class _AttnCore(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, cos, sin, T, S, K, H, pattern):
        qkv = qkv.contiguous()
        B, n = qkv.shape[0], qkv.shape[1]
        col = pattern == PATTERN_IDS["axial_col"]
        q, k, v = C().rope_fwd(qkv, cos, sin, T, S, H, col, 0.125)
        out, lse = C().attn_fwd(q, k, v, B, T, S, n, K, H, pattern)
        ctx.save_for_backward(q, k, v, out, lse, cos, sin)
        ctx.geo = (B, T, S, n, K, H, pattern, col)
        return out

    @staticmethod
    def backward(ctx, gout):
        q, k, v, out, lse, cos, sin = ctx.saved_tensors
        B, T, S, n, K, H, pattern, col = ctx.geo
        gout = gout.to(torch.bfloat16).contiguous()
        dqkv = C().attn_bwd_rope(q, k, v, out, gout, lse, cos, sin, B, T, S, n, K, H, pattern, 0.125, *_rot_freqs(q.device))
        return dqkv, None, None, None, None, None, None, None


def attention_core(qkv, heads: int, geom: AttnGeometry, attn_type: str):
    dim_head = qkv.shape[-1] // 3 // heads
    assert dim_head == 64, "the HIP attention kernels are specialised for dim_head = 64"
    cos, sin = _rope_tables(geom, dim_head, qkv.device)
    return _AttnCore.apply(qkv, cos, sin, geom.text_len, geom.image_size, geom.kernel_size, heads, PATTERN_IDS[attn_type])


def attention_out(h, w_qkv, heads: int, geom: AttnGeometry, attn_type: str):
    """QKV GEMM -> rotary -> sparse attention; returns the pre-projection output (B, n, H*64)."""
    return attention_core(linear(h, w_qkv), heads, geom, attn_type)


def attention_block(h, w_qkv, w_out, b_out, heads: int, geom: AttnGeometry, attn_type: str):
    return linear(attention_out(h, w_qkv, heads, geom, attn_type), w_out, b_out)


# ---------------------------------------------------------------------------------------------
# Whole pre-norm sublayers, x -> x + LayerScale * branch(LN_shift(x)), as ONE autograd node each with
# a hand-written backward (reference: dalle_pytorch/transformer.py PreNorm / PreShiftToken /
# LayerScale around Attention and FeedForward). Versus chaining the per-op Functions this removes the
# residual-grad add (it happens inside the LN-backward kernel) and, with the flat grad arena, every
# parameter-grad add: GEMM weight grads accumulate in hipBLASLt (beta = 1), LayerNorm / LayerScale /
# bias grads accumulate inside the column-reduction kernel.
# ---------------------------------------------------------------------------------------------
def _sinks(params, needs):
    """Arena grad buffers for every parameter, or None if any needed one is missing (fallback: return
    all grads to autograd)."""
    sinks = [grad_sink(p) for p in params]
    if all(n for n in needs) and all(s is not None for s in sinks):
        return sinks
    return None


# Each sublayer = LN_shift (prologue) -> core (projections, attention / GEGLU) -> LayerScale residual
# (epilogue). The cores are shared by the per-sublayer autograd nodes, the reversible stack and the
# sequential stack, which fuses each epilogue with the NEXT sublayer's prologue (ln_shift_fwd_res /
# ln_shift_bwd_sr).
def _attn_core_fwd(inp, h, mean, rstd, w_qkv, w_out, b_out, scale, cos, sin, meta, save: bool = True):
    """to_out(attn(rope(to_qkv(h)))) + b_out (bf16, pre-LayerScale) and the saved tensors."""
    T, S, K, H, pattern, shift = meta
    B, n, d = inp.shape
    h2 = h.view(-1, d)
    wq = bf16_weight(w_qkv)
    col = pattern == PATTERN_IDS["axial_col"]
    if ASM_GEMM and n % 256 == 0 and asm_fused_k(d) and wq.shape[0] == 3 * H * 64 and (H * 64) % 256 == 0 and h2.stride(1) == 1:
        # QKV GEMM on the assembly kernel, the rotary applied to its stored bf16 values in the deferred epilogue
        q, k, v = C().asm_qkv_rope(h2, wq, _cs3_from_tables(cos, sin, 0.125), T, S, H, n, col)
        _count("qkv_rope")
        _count("asm_qkv_rope")
    elif (B * n) % 256 == 0 and wq.shape[0] % 256 == 0 and d % 64 == 0 and d >= 128:
        # QKV GEMM with the rotary fused into its epilogue: writes the attention storage directly
        q, k, v = C().qkv_rope_pt(h2, wq, _cs_from_tables(cos, sin), T, S, H, n, col, 0.125)
        _count("qkv_rope")
    else:
        qkv = torch.mm(h2, wq.t()).view(B, n, -1)
        q, k, v = C().rope_fwd(qkv, cos, sin, T, S, H, col, 0.125)
        del qkv
    out, lse = C().attn_fwd(q, k, v, B, T, S, n, K, H, pattern)
    wo = bf16_weight(w_out)
    y = mm_nt(out.view(-1, out.shape[-1]), wo, b_out)
    s = scale.reshape(-1).contiguous()
    if not save:
        return y, s, None
    h2 = saved_gemm_input(h2)  # the QKV weight grad's input, token-contiguous
    return y, s, (inp, mean, rstd, h2, wq, q, k, v, out, lse, y, wo, s, cos, sin, (B, n, T, S, K, H, pattern, shift, col))


def _attn_core_bwd(saved, params, dy):
    """dy (bf16, grad of the pre-LayerScale output) -> dh (grad of the LN output) + (dw_qkv, dw_out)."""
    x, mean, rstd, h2, wq, q, k, v, out, lse, y, wo, s, cos, sin, geo = saved
    ln_w, ln_b, w_qkv, w_out, b_out, scale = params
    B, n, T, S, K, H, pattern, shift, col = geo
    dy = dy.view(-1, dy.shape[-1])
    o2 = out.view(-1, out.shape[-1])
    do = input_grad(dy, w_out).view(out.shape)
    dwo = weight_grad(w_out, dy, o2)
    # rotary backward inside the attention-backward epilogues
    dqkv = C().attn_bwd_rope(q, k, v, out, do, lse, cos, sin, B, T, S, n, K, H, pattern, 0.125,
                             *_rot_freqs(q.device)).view(B * n, -1)
    del do
    dh = input_grad(dqkv, w_qkv).view(x.shape)
    dwq = weight_grad(w_qkv, dqkv, h2)
    return dh, dwq, dwo


def _ff_core_fwd(inp, h, mean, rstd, w1, b1, w2, b2, scale, meta, save: bool = True):
    """W2 GEGLU(W1 h + b1) + b2 (bf16, pre-LayerScale) and the saved tensors."""
    d = inp.shape[-1]
    h2 = h.view(-1, d)
    w1b, w2b = bf16_weight(w1), bf16_weight(w2)
    if b1 is not None and _ff_in_geglu_ok(h2, w1):
        a, u = ff_in_geglu(h2, w1, b1)
    else:
        a = mm_nt(h2, w1b, b1)
        u = C().geglu_fwd(a)
    if not save:
        del a
    y = mm_nt(u, w2b, b2)
    s = scale.reshape(-1).contiguous()
    if not save:
        return y, s, None
    h2 = saved_gemm_input(h2)  # the FF-in weight grad's input, token-contiguous
    return y, s, (inp, mean, rstd, h2, w1b, a, u, w2b, y, s, meta)


def _ff_core_bwd(saved, params, dy, sk):
    """Same contract as ``_attn_core_bwd``; the FF-in bias grad goes to sink ``sk[3]`` when given."""
    x, mean, rstd, h2, w1b, a, u, w2b, y, s, meta = saved
    ln_w, ln_b, w1, b1, w2, b2, scale = params
    dy = dy.view(-1, dy.shape[-1])
    M, F = dy.shape[0], w2b.shape[1]
    if ASM_GEMM and M % 256 == 0 and F % 256 == 0 and asm_fused_k(dy.shape[1]) and dy.stride(1) == 1:
        # du = dy W2 on the assembly GEMM, the GEGLU backward + b1 column sums under the next tile's K-steps
        da, db1 = C().asm_ff_dgrad_geglu(dy, bf16_weight_t(w2), a.view(M, 2 * F), sk[3] if sk is not None else None)
        _count("ff_dgrad_geglu")
        _count("asm_ff_dgrad_geglu")
        dw2 = weight_grad(w2, saved_gemm_input(dy, WGRAD_GT), u)
    elif M % 256 == 0 and F % 256 == 0 and dy.shape[1] % 64 == 0:
        # du = dy W2 on the hand-written GEMM with the GEGLU backward + b1 grad in its epilogue
        da, db1 = C().ff_dgrad_geglu(dy, bf16_weight_t(w2), a.view(M, 2 * F), sk[3] if sk is not None else None)
        _count("ff_dgrad_geglu")
        dw2 = weight_grad(w2, saved_gemm_input(dy, WGRAD_GT), u)
    else:
        du = input_grad(dy, w2)
        dw2 = weight_grad(w2, dy, u)
        da, db1 = C().geglu_bwd_bias(a, du, sk[3] if sk is not None else None)
        del du
    dh = input_grad(da, w1).view(x.shape)
    dw1 = weight_grad(w1, da, h2)
    return dh, dw1, db1, dw2


def _attn_fwd(res, inp, ln_w, ln_b, w_qkv, w_out, b_out, scale, cos, sin, meta, save: bool, sign: float = 1.0):
    """res + sign * scale * to_out(attn(rope(to_qkv(LN_shift(inp))))); returns (out, saved-or-None)."""
    T, S, K, H, pattern, shift = meta
    inp = inp.contiguous()
    h, mean, rstd = C().ln_shift_fwd(inp, ln_w.contiguous(), ln_b.contiguous(), T, S, shift, 1e-5)
    y, s, saved = _attn_core_fwd(inp, h, mean, rstd, w_qkv, w_out, b_out, scale, cos, sin, meta, save)
    xo = torch.empty_like(res)
    C().scale_residual_out(res.contiguous(), y, s if sign > 0 else -s, xo)
    return xo, saved


def _residual_bwd(g, y, s, scale, sk, i_scale, i_bias):
    """LayerScale-residual backward: dy = bf16(s * g); dscale / dbias to the sinks or returned."""
    if sk is not None:
        dy, _, _ = C().scale_residual_bwd(g, y, s, sk[i_scale], sk[i_bias])
        return dy, None, None
    dy, dscale, gsum = C().scale_residual_bwd(g, y, s)
    return dy, gsum * s, dscale.view(scale.shape)


def _ln_bwd(x, ln_w, dh, mean, rstd, meta_ln, resid, sk):
    T, S, shift = meta_ln
    resid = resid.contiguous() if resid is not None else None
    if sk is not None:
        return C().ln_shift_bwd(x, ln_w.contiguous(), dh, mean, rstd, T, S, shift, resid, sk[0], sk[1])
    return C().ln_shift_bwd(x, ln_w.contiguous(), dh, mean, rstd, T, S, shift, resid)


def _attn_bwd(saved, params, needs, g, resid):
    """Backward of ``_attn_fwd`` for the branch upstream grad ``g`` (fp32): returns (d inp + resid,
    dln_w, dln_b, dw_qkv, dw_out, db_out, dscale); the parameter grads are None when they went to the
    arena sinks. ``resid`` (fp32, may be None) is added to d inp inside the LayerNorm-backward kernel."""
    x, mean, rstd, geo = saved[0], saved[1], saved[2], saved[15]
    sk = _sinks(params, needs)
    dy, db, dscale = _residual_bwd(g.contiguous(), saved[10], saved[12], params[5], sk, 5, 4)
    dh, dwq, dwo = _attn_core_bwd(saved, params, dy)
    dx, dlw, dlb = _ln_bwd(x, params[0], dh, mean, rstd, (geo[2], geo[3], geo[7]), resid, sk)
    return dx, dlw, dlb, dwq, dwo, db, dscale


def _ff_fwd(res, inp, ln_w, ln_b, w1, b1, w2, b2, scale, meta, save: bool, sign: float = 1.0):
    """res + sign * scale * (W2 GEGLU(W1 LN_shift(inp) + b1) + b2); returns (out, saved-or-None)."""
    T, S, shift = meta
    inp = inp.contiguous()
    h, mean, rstd = C().ln_shift_fwd(inp, ln_w.contiguous(), ln_b.contiguous(), T, S, shift, 1e-5)
    y, s, saved = _ff_core_fwd(inp, h, mean, rstd, w1, b1, w2, b2, scale, meta, save)
    xo = torch.empty_like(res)
    C().scale_residual_out(res.contiguous(), y, s if sign > 0 else -s, xo)
    return xo, saved


def _ff_bwd(saved, params, needs, g, resid):
    """Backward of ``_ff_fwd`` (same contract as ``_attn_bwd``)."""
    x, mean, rstd, meta = saved[0], saved[1], saved[2], saved[10]
    sk = _sinks(params, needs)
    dy, db2, dscale = _residual_bwd(g.contiguous(), saved[8], saved[9], params[6], sk, 6, 5)
    dh, dw1, db1, dw2 = _ff_core_bwd(saved, params, dy, sk)
    dx, dlw, dlb = _ln_bwd(x, params[0], dh, mean, rstd, meta, resid, sk)
    return dx, dlw, dlb, dw1, db1, dw2, db2, dscale


def _ln_spec(args, kind):
    """(ln_w, ln_b, (T, S, shift)) of a reversible block's sublayer argument tuple."""
    if kind == "attn":
        meta = args[8]
        return args[0], args[1], (meta[0], meta[1], meta[5])
    return args[0], args[1], args[7]


def _residual_chain(res, y, s, sign, nxt):
    """res + sign * s * y (fp32) and, when ``nxt`` (the LN spec of the sublayer that reads it) is given, its
    LayerNorm(+shift) in the same kernel (ln_shift_fwd_res: one read of the residual stream instead of two)."""
    s = s if sign > 0 else -s
    if nxt is None:
        xo = torch.empty_like(res)
        C().scale_residual_out(res.contiguous(), y, s, xo)
        return xo, None
    nw, nb, (T, S, shift) = nxt
    xo, h, mean, rstd = C().ln_shift_fwd_res(res.contiguous(), y, s, nw.contiguous(), nb.contiguous(), T, S, shift, 1e-5)
    return xo, (h, mean, rstd)


def _attn_step(res, inp, args, pre, nxt, save: bool, sign: float = 1.0):
    """``_attn_fwd`` whose LayerNorm may come precomputed (``pre`` = (h, mean, rstd) of ``inp``, from the
    residual kernel that produced it) and whose residual update may carry the next sublayer's LayerNorm
    (``nxt``). Returns (out, saved-or-None, LN of out or None)."""
    ln_w, ln_b, w_qkv, w_out, b_out, scale, cos, sin, meta = args
    T, S, K, H, pattern, shift = meta
    inp = inp.contiguous()
    h, mean, rstd = pre if pre is not None else C().ln_shift_fwd(inp, ln_w.contiguous(), ln_b.contiguous(), T, S, shift, 1e-5)
    y, s, saved = _attn_core_fwd(inp, h, mean, rstd, w_qkv, w_out, b_out, scale, cos, sin, meta, save)
    xo, ln_next = _residual_chain(res, y, s, sign, nxt)
    return xo, saved, ln_next


def _ff_step(res, inp, args, pre, nxt, save: bool, sign: float = 1.0):
    """``_ff_fwd`` with the same LayerNorm hand-over as ``_attn_step``."""
    ln_w, ln_b, w1, b1, w2, b2, scale, meta = args
    T, S, shift = meta
    inp = inp.contiguous()
    h, mean, rstd = pre if pre is not None else C().ln_shift_fwd(inp, ln_w.contiguous(), ln_b.contiguous(), T, S, shift, 1e-5)
    y, s, saved = _ff_core_fwd(inp, h, mean, rstd, w1, b1, w2, b2, scale, meta, save)
    xo, ln_next = _residual_chain(res, y, s, sign, nxt)
    return xo, saved, ln_next


def _rev_sub_bwd(kind, saved, params, sk, g, resid, dy=None, prev=None):
    """Reversible-stack sublayer backward on the arena sinks ``sk``. ``dy`` (bf16 grad of the pre-LayerScale
    output) is either given -- the previous LN backward produced it -- or computed from the residual grad
    ``g``; the LN backward adds ``resid`` into dx and, with ``prev`` = (y_prev, s_prev, dscale sink, dbias
    sink) of the sublayer that produced this one's LN input, also runs that sublayer's LayerScale-residual
    backward in the same kernel (ln_shift_bwd_sr). Returns (dx, dy_prev or None)."""
    i_s, i_b = _SCALE_BIAS[kind]
    if dy is None:
        y, s = (saved[10], saved[12]) if kind == "attn" else (saved[8], saved[9])
        dy, _, _ = C().scale_residual_bwd(g.contiguous(), y, s, sk[i_s], sk[i_b])
    if kind == "attn":
        dh, _, _ = _attn_core_bwd(saved, params, dy)
        geo = saved[15]
        T, S, shift = geo[2], geo[3], geo[7]
    else:
        dh, _, _, _ = _ff_core_bwd(saved, params, dy, sk)
        T, S, shift = saved[10]
    x, mean, rstd = saved[0], saved[1], saved[2]
    if prev is None:
        dx, _, _ = C().ln_shift_bwd(x, params[0].contiguous(), dh, mean, rstd, T, S, shift, resid.contiguous(), sk[0], sk[1])
        return dx, None
    yp, sp, gsp, gbp = prev
    dx, dyp = C().ln_shift_bwd_sr(x, params[0].contiguous(), dh, mean, rstd, T, S, shift, resid.contiguous(), yp, sp,
                                  sk[0], sk[1], gsp, gbp)
    return dx, dyp


def _res_of(kind, saved, sk):
    """(y, s, dscale sink, dbias sink) of a sublayer's LayerScale residual, for ``_rev_sub_bwd(prev=...)``."""
    i_s, i_b = _SCALE_BIAS[kind]
    y, s = (saved[10], saved[12]) if kind == "attn" else (saved[8], saved[9])
    return y, s, sk[i_s], sk[i_b]


class _AttnSublayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ln_w, ln_b, w_qkv, w_out, b_out, scale, cos, sin, meta):
        xo, saved = _attn_fwd(x, x, ln_w, ln_b, w_qkv, w_out, b_out, scale, cos, sin, meta, save=True)
        ctx.saved = saved
        ctx.params = (ln_w, ln_b, w_qkv, w_out, b_out, scale)
        return xo

    @staticmethod
    def backward(ctx, g):
        saved, ctx.saved = ctx.saved, None
        g = g.contiguous()
        grads = _attn_bwd(saved, ctx.params, ctx.needs_input_grad[1:7], g, g)
        return (*grads, None, None, None)


class _FFSublayer(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ln_w, ln_b, w1, b1, w2, b2, scale, meta):
        xo, saved = _ff_fwd(x, x, ln_w, ln_b, w1, b1, w2, b2, scale, meta, save=True)
        ctx.saved = saved
        ctx.params = (ln_w, ln_b, w1, b1, w2, b2, scale)
        return xo

    @staticmethod
    def backward(ctx, g):
        saved, ctx.saved = ctx.saved, None
        g = g.contiguous()
        grads = _ff_bwd(saved, ctx.params, ctx.needs_input_grad[1:8], g, g)
        return (*grads, None)


# ---------------------------------------------------------------------------------------------
# Reversible stack over the fused sublayers. Forward: y1 = x1 + f(x2),
# y2 = x2 + g(y1) with nothing saved but the final (y1, y2). Backward per block, newest first:
#   x2 = y2 - g(y1)  (the fused FF sublayer run with sign -1, saving its activations)
#   dy1 += g'(y1)^T dy2   (its hand-written backward; the residual add happens inside the LN-bwd kernel)
#   x1 = y1 - f(x2); dy2 += f'(x2)^T dy1   (same with the attention sublayer)
# so the recompute costs exactly one forward per block and no autograd graph is built.
# ---------------------------------------------------------------------------------------------
REV_STATS: Dict[str, float] = {}  # last reversible forward: blocks kept / total / bytes kept ("auto" only)


def rev_store_budget(device) -> float:
    """Bytes of block activations the reversible stack may keep from the forward ("auto" policy): what
    the device can still hold -- free HBM plus the caching allocator's idle reserve -- minus a margin
    for the backward's own working set (max(6 GB, 8 % of HBM)). ``DALLE_AMD_REV_STORE_GB`` overrides."""
    env = os.environ.get("DALLE_AMD_REV_STORE_GB")
    if env is not None:
        return float(env) * 2 ** 30
    if device.type != "cuda":
        return 0.0
    free, total = torch.cuda.mem_get_info(device)
    idle = torch.cuda.memory_reserved(device) - torch.cuda.memory_allocated(device)
    return max(0.0, free + idle - max(6 * 2 ** 30, 0.08 * total))


# ---------------------------------------------------------------------------------------------
# Data-parallel hand-off: the fused stacks' backward reports parameters whose arena grads just became
# final (their last use in backward order), so the gradient all-reduce of those ranges can start while
# the remaining layers' backward runs (parallel/dp.py GradSync.attach).
# ---------------------------------------------------------------------------------------------
_grad_ready_hook = None


def set_grad_ready_hook(fn):
    global _grad_ready_hook
    prev, _grad_ready_hook = _grad_ready_hook, fn
    return prev


def _final_at(groups):
    """``groups[i]`` = params used by step i (forward order); returns, per step, the params whose LAST
    use in backward order (descending i) is step i -- i.e. whose first forward use is i."""
    first = {}
    for i, prm in enumerate(groups):
        for p in prm:
            first.setdefault(id(p), i)
    out = [[] for _ in groups]
    seen = set()
    for i, prm in enumerate(groups):
        for p in prm:
            if first[id(p)] == i and id(p) not in seen:
                seen.add(id(p))
                out[i].append(p)
    return out


class _ReversibleFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, blocks, recompute, *params):
        """``recompute``: True rebuilds every block in backward, False keeps every block's activations,
        "auto" keeps the FIRST blocks' activations while they fit rev_store_budget (the backward, newest
        block first, rebuilds the rest from the outputs and then runs on the stored ones)."""
        _count("reversible_stack")
        x1 = x2 = x.contiguous()
        if recompute == "auto":
            budget = rev_store_budget(x.device)
        else:
            budget = 0.0 if recompute else float("inf")
        stored, used, storing = [], 0.0, budget > 0
        cuda = x.is_cuda
        with torch.no_grad():
            pre = None  # LN of x2 for the next attention sublayer, computed by the residual kernel that wrote x2
            for bi, (fa, ga) in enumerate(blocks):
                before = torch.cuda.memory_allocated(x.device) if (cuda and storing and budget != float("inf")) else 0
                nxt = _ln_spec(blocks[bi + 1][0][0], "attn") if bi + 1 < len(blocks) else None
                x1, sf, pre_g = _attn_step(x1, x2, fa[0], pre, _ln_spec(ga[0], "ff"), save=storing)
                x2, sg, pre = _ff_step(x2, x1, ga[0], pre_g, nxt, save=storing)
                del pre_g
                if storing:
                    if budget != float("inf") and cuda:
                        # this block's retained bytes; keep a second block's worth free for the backward
                        delta = torch.cuda.memory_allocated(x.device) - before
                        if used + 2 * delta > budget:
                            del sf, sg
                            storing = False
                            continue
                        used += delta
                    stored.append((sf, sg))
        REV_STATS.update(stored=len(stored), blocks=len(blocks), stored_bytes=used)
        ctx.blocks = blocks
        ctx.params = params
        ctx.stored = stored
        ctx.save_for_backward(x1, x2)
        return (x1 + x2) * 0.5

    @staticmethod
    def backward(ctx, gout):
        y1, y2 = ctx.saved_tensors
        blocks = ctx.blocks
        dy1 = dy2 = (gout.float() * 0.5).contiguous()
        pending: Dict[int, torch.Tensor] = {}  # grads that found no arena sink, keyed by id(param)

        def collect(plist, grads):
            for p, gr in zip(plist, grads):
                if gr is None:
                    continue
                k = id(p)
                pending[k] = gr if k not in pending else pending[k] + gr

        stored, ctx.stored = ctx.stored, None
        hook = _grad_ready_hook
        final = _final_at([fa[1] + ga[1] for fa, ga in blocks]) if hook is not None else None
        sinks = [(_sinks(fa[1], [p.requires_grad for p in fa[1]]), _sinks(ga[1], [p.requires_grad for p in ga[1]]))
                 for fa, ga in blocks]
        if all(a is not None and b is not None for a, b in sinks):
            dx = _ReversibleFused._backward_chained(blocks, stored, sinks, y1, y2, dy1, dy2, hook, final)
            return (dx, None, None, *([None] * len(ctx.params)))
        with torch.no_grad():
            for bi in reversed(range(len(blocks))):
                fa, ga = blocks[bi]
                g_args, g_params = ga
                f_args, f_params = fa
                rebuild = bi >= len(stored)  # blocks past the stored prefix are rebuilt from their outputs
                if rebuild:
                    # x2 = y2 - g(y1), with f's LayerNorm of x2 from the same residual kernel
                    x2, saved_g, pre_f = _ff_step(y2, y1, g_args, None, _ln_spec(f_args, "attn"), save=True, sign=-1.0)
                else:
                    saved_f, saved_g = stored.pop()
                res = _ff_bwd(saved_g, g_params, [p.requires_grad for p in g_params], dy2, dy1)
                del saved_g
                dy1 = res[0]
                collect(g_params, res[1:])
                if rebuild:
                    x1, saved_f, _ = _attn_step(y1, x2, f_args, pre_f, None, save=True, sign=-1.0)
                    del pre_f
                    y1, y2 = x1, x2
                res = _attn_bwd(saved_f, f_params, [p.requires_grad for p in f_params], dy1, dy2)
                del saved_f
                dy2 = res[0]
                collect(f_params, res[1:])
                if final is not None and final[bi]:
                    hook([p for p in final[bi] if id(p) not in pending])
        dx = dy1 + dy2
        return (dx, None, None, *[pending.get(id(p)) for p in ctx.params])

    @staticmethod
    def _backward_chained(blocks, stored, sinks, y1, y2, dy1, dy2, hook, final):
        """Backward with every parameter grad in the arena and each LayerScale-residual backward fused into
        the LayerNorm backward that produces its input grad (ln_shift_bwd_sr), as in the sequential stack:
        g's LN backward (-> dy1) also yields f's dy; f's LN backward (-> dy2) also yields the PREVIOUS
        block's g dy. So a block's f is rebuilt before g's backward, and the previous block's g one step
        ahead (one more sublayer's activations alive at a time)."""
        L = len(blocks)
        ahead = None   # (x2, saved_g, pre_f) of the next block to process, rebuilt early
        dyg = None     # g's dy of the block being processed, produced by the later block's f LN backward
        with torch.no_grad():
            for bi in reversed(range(L)):
                fa, ga = blocks[bi]
                f_args, f_params = fa
                g_args, g_params = ga
                sk_f, sk_g = sinks[bi]
                rebuild = bi >= len(stored)
                if rebuild:
                    if ahead is not None:
                        x2, saved_g, pre_f = ahead
                        ahead = None
                    else:
                        x2, saved_g, pre_f = _ff_step(y2, y1, g_args, None, _ln_spec(f_args, "attn"), save=True, sign=-1.0)
                    # x1 = y1 - f(x2), with the previous block's g LayerNorm of x1 from the same kernel
                    nxt_g = _ln_spec(blocks[bi - 1][1][0], "ff") if bi > 0 and bi - 1 >= len(stored) else None
                    x1, saved_f, pre_gp = _attn_step(y1, x2, f_args, pre_f, nxt_g, save=True, sign=-1.0)
                    del pre_f
                else:
                    saved_f, saved_g = stored.pop()
                    pre_gp = None
                # g: LN backward adds dy1 and yields f's dy
                dy1, dyf = _rev_sub_bwd("ff", saved_g, g_params, sk_g, dy2, dy1, dy=dyg,
                                        prev=_res_of("attn", saved_f, sk_f))
                del saved_g
                # the previous block's g (its residual consumes f's input grad dy2)
                prev = None
                if bi > 0:
                    pf_args, _ = blocks[bi - 1][0]
                    pg_args, _ = blocks[bi - 1][1]
                    psk_g = sinks[bi - 1][1]
                    if bi - 1 >= len(stored):  # rebuilt: x2_prev = x2 - g_prev(x1), f_prev's LN on the way
                        ahead = _ff_step(x2, x1, pg_args, pre_gp, _ln_spec(pf_args, "attn"), save=True, sign=-1.0)
                        prev = _res_of("ff", ahead[1], psk_g)
                    else:
                        prev = _res_of("ff", stored[-1][1], psk_g)
                pre_gp = None
                dy2, dyg = _rev_sub_bwd("attn", saved_f, f_params, sk_f, dy1, dy2, dy=dyf, prev=prev)
                del saved_f
                if rebuild:
                    y1, y2 = x1, x2
                if final is not None and final[bi]:
                    hook(final[bi])
        return dy1 + dy2


def reversible_stack(x, layers, geom: AttnGeometry, text_len: int, image_size: int, recompute=True):
    """``layers``: per block ((ln_w, ln_b, w_qkv, w_out, b_out, scale, heads, attn_type, shift),
    (ln_w, ln_b, w1, b1, w2, b2, scale, shift)). Returns mean(y1, y2) of the reversible stack.
    ``recompute=False`` keeps every block's activations from the forward instead of rebuilding them
    in backward (same coupling math; one forward less per step for ~depth x the activation memory);
    ``"auto"`` keeps as many blocks as the HBM left over holds (see _ReversibleFused.forward)."""
    blocks, uniq, seen = [], [], set()
    for (aln_w, aln_b, w_qkv, w_out, b_out, ascale, heads, attn_type, ashift), (fln_w, fln_b, w1, b1, w2, b2, fscale, fshift) in layers:
        dim_head = w_qkv.shape[0] // 3 // heads
        assert dim_head == 64, "the HIP attention kernels are specialised for dim_head = 64"
        cos, sin = _rope_tables(geom, dim_head, x.device)
        ameta = (geom.text_len, geom.image_size, geom.kernel_size, heads, PATTERN_IDS[attn_type], bool(ashift))
        aparams = (aln_w, aln_b, w_qkv, w_out, b_out, ascale)
        fparams = (fln_w, fln_b, w1, b1, w2, b2, fscale)
        blocks.append((((*aparams, cos, sin, ameta), aparams),
                       ((*fparams, (text_len, image_size, bool(fshift))), fparams)))
        for p in aparams + fparams:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
    return _ReversibleFused.apply(x, blocks, recompute if recompute == "auto" else bool(recompute), *uniq)


# ---------------------------------------------------------------------------------------------
# Sequential (non-reversible) stack as ONE autograd node: every sublayer boundary runs as a single
# kernel -- forward x_{i+1} = x_i + s_i * y_i fused with LN_shift_{i+1}(x_{i+1}) (ln_shift_fwd_res),
# backward LN_shift_{i+1}' + residual fused with sublayer i's LayerScale backward (ln_shift_bwd_sr)
# -- so the fp32 residual stream is read once per boundary in each direction instead of twice.
# Parameter grads go straight to the flat-arena sinks (required; otherwise the per-sublayer nodes run).
# ---------------------------------------------------------------------------------------------

# per sublayer kind: (index of the LayerScale param, of the output-projection bias) in its param tuple
_SCALE_BIAS = {"attn": (5, 4), "ff": (6, 5)}


def _ln_meta(kind, args):
    """(text_len, image_size, shift) of a sublayer's LN-shift prologue."""
    m = args[-1]
    return (m[0], m[1], m[5]) if kind == "attn" else m


class _SequentialFused(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, subs, *params):
        _count("sequential_stack")
        x = x.contiguous()
        saved_all = []
        kind, args, prm = subs[0]
        T, S, shift = _ln_meta(kind, args)
        h, mean, rstd = C().ln_shift_fwd(x, prm[0].contiguous(), prm[1].contiguous(), T, S, shift, 1e-5)
        inp = x
        for i, (kind, args, prm) in enumerate(subs):
            if kind == "attn":
                y, s, saved = _attn_core_fwd(inp, h, mean, rstd, *prm[2:], *args[-3:])
            else:
                y, s, saved = _ff_core_fwd(inp, h, mean, rstd, *prm[2:], args[-1])
            saved_all.append(saved)
            if i + 1 < len(subs):
                nkind, nargs, nprm = subs[i + 1]
                T, S, shift = _ln_meta(nkind, nargs)
                inp, h, mean, rstd = C().ln_shift_fwd_res(inp, y, s, nprm[0].contiguous(), nprm[1].contiguous(), T, S, shift,
                                                          1e-5)
            else:
                out = torch.empty_like(inp)
                C().scale_residual_out(inp, y, s, out)
        ctx.subs, ctx.saved_all, ctx.params = subs, saved_all, params
        return out

    @staticmethod
    def backward(ctx, gout):
        subs, saved_all = ctx.subs, ctx.saved_all
        ctx.saved_all = None
        # The forward chose this node because every parameter had an fp32 grad buffer. If they were reset
        # since (``loss = model(x); opt.zero_grad(); loss.backward()``), give them fresh zero fp32 .grad
        # buffers: every kernel and weight-grad GEMM below accumulates into .grad, exactly as into the arena
        reset = False
        for p in ctx.params:
            if p.requires_grad and grad_sink(p) is None:
                p.grad = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.contiguous_format)
                reset = True
        sinks = [[grad_sink(p) for p in prm] for _, _, prm in subs]
        g = gout.float().contiguous()
        g = _SequentialFused._backward(subs, saved_all, sinks, g, handoff=not reset)
        return (g, None, *([None] * len(ctx.params)))

    @staticmethod
    def _backward(subs, saved_all, sinks, g, handoff: bool = True):
        hook = _grad_ready_hook if handoff else None
        final = _final_at([prm for _, _, prm in subs]) if hook is not None else None
        with torch.no_grad():
            kind, args, prm = subs[-1]
            i_s, i_b = _SCALE_BIAS[kind]
            sv = saved_all[-1]
            y, s = (sv[10], sv[12]) if kind == "attn" else (sv[8], sv[9])
            dy, _, _ = C().scale_residual_bwd(g, y, s, sinks[-1][i_s], sinks[-1][i_b])
            for i in range(len(subs) - 1, -1, -1):
                kind, args, prm = subs[i]
                sv = saved_all[i]
                saved_all[i] = None
                sk = sinks[i]
                if kind == "attn":
                    dh, _, _ = _attn_core_bwd(sv, prm, dy)
                else:
                    dh, _, _, _ = _ff_core_bwd(sv, prm, dy, sk)
                x, mean, rstd = sv[0], sv[1], sv[2]
                T, S, shift = _ln_meta(kind, args)
                if i > 0:
                    pkind, _, _ = subs[i - 1]
                    ps_, pb_ = _SCALE_BIAS[pkind]
                    pv = saved_all[i - 1]
                    yp, sp = (pv[10], pv[12]) if pkind == "attn" else (pv[8], pv[9])
                    g, dy = C().ln_shift_bwd_sr(x, prm[0].contiguous(), dh, mean, rstd, T, S, shift, g, yp, sp, sk[0], sk[1],
                                                sinks[i - 1][ps_], sinks[i - 1][pb_])
                else:
                    g, _, _ = C().ln_shift_bwd(x, prm[0].contiguous(), dh, mean, rstd, T, S, shift, g, sk[0], sk[1])
                del sv
                # sublayer i's LayerScale / bias grads were written one iteration earlier (its successor's
                # LN backward), its weights and LN grads just now
                if final is not None and final[i]:
                    hook(final[i])
        return g


def attn_args(x, w_qkv, heads: int, geom: AttnGeometry, attn_type: str, shift: bool):
    dim_head = w_qkv.shape[0] // 3 // heads
    assert dim_head == 64, "the HIP attention kernels are specialised for dim_head = 64"
    cos, sin = _rope_tables(geom, dim_head, x.device)
    return (heads, cos, sin, (geom.text_len, geom.image_size, geom.kernel_size, heads, PATTERN_IDS[attn_type], bool(shift)))


def sequential_stack(x, subs):
    """``subs``: per sublayer ("attn", (heads, cos, sin, meta), (ln_w, ln_b, w_qkv, w_out, b_out, scale)) or
    ("ff", (meta,), (ln_w, ln_b, w1, b1, w2, b2, scale)). Returns None when some parameter has no fp32
    arena grad buffer (the caller then runs the per-sublayer nodes)."""
    uniq, seen = [], set()
    for _, _, prm in subs:
        for p in prm:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
    if not FUSE_WGRAD or any(not p.requires_grad or grad_sink(p) is None for p in uniq):
        return None
    return _SequentialFused.apply(x, subs, *uniq)


def attn_sublayer(x, ln_w, ln_b, w_qkv, w_out, b_out, scale, heads: int, geom: AttnGeometry, attn_type: str, shift: bool):
    """x + scale * to_out(sparse_attention(rotary(to_qkv(LN_shift(x))))) in one autograd node."""
    dim_head = w_qkv.shape[0] // 3 // heads
    assert dim_head == 64, "the HIP attention kernels are specialised for dim_head = 64"
    cos, sin = _rope_tables(geom, dim_head, x.device)
    meta = (geom.text_len, geom.image_size, geom.kernel_size, heads, PATTERN_IDS[attn_type], bool(shift))
    return _AttnSublayer.apply(x, ln_w, ln_b, w_qkv, w_out, b_out, scale, cos, sin, meta)


def ff_sublayer(x, ln_w, ln_b, w1, b1, w2, b2, scale, text_len: int, image_size: int, shift: bool):
    """x + scale * W2 GEGLU(W1 LN_shift(x) + b1) + b2 in one autograd node."""
    return _FFSublayer.apply(x, ln_w, ln_b, w1, b1, w2, b2, scale, (text_len, image_size, bool(shift)))


# ---------------------------------------------------------------------------------------------
# K9: GEGLU feed-forward
# ---------------------------------------------------------------------------------------------
class _GEGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h):
        h = h.contiguous()
        ctx.save_for_backward(h)
        return C().geglu_fwd(h)

    @staticmethod
    def backward(ctx, g):
        (h,) = ctx.saved_tensors
        return C().geglu_bwd(h, g.to(torch.bfloat16).contiguous())


def feed_forward(h, w1, b1, w2, b2):
    return linear(_FF1GEGLU.apply(h, w1, b1), w2, b2)


# ---------------------------------------------------------------------------------------------
# K8/K10 epilogue: x + scale * y (fp32 residual stream)
# ---------------------------------------------------------------------------------------------
class _ScaleResidual(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, scale):
        out = x.contiguous().clone()
        y = y.contiguous()
        s = scale.reshape(-1).contiguous()
        C().scale_residual_(out, y, s)
        ctx.save_for_backward(y, s)
        ctx.sshape = scale.shape
        return out

    @staticmethod
    def backward(ctx, g):
        y, s = ctx.saved_tensors
        dy, ds, _ = C().scale_residual_bwd(g.contiguous(), y, s)
        return g, dy, ds.view(ctx.sshape)


def scale_residual(x, y, scale):
    return _ScaleResidual.apply(x, y, scale)


# ---------------------------------------------------------------------------------------------
# K12: final LayerNorm + split-vocabulary logits + fused softmax cross entropy
# ---------------------------------------------------------------------------------------------
class _SplitXent(torch.autograd.Function):
    """K12: final-LN output -> split-vocabulary logits (text rows x 32356 text columns, image rows x 8192
    image columns: the static logits mask makes every other column -inf, so it is skipped exactly) ->
    fused log-softmax + NLL, loss = (CE_text + w * CE_img) / (1 + w).

    Logits are never materialised for the whole batch: the rows are processed in chunks of
    ``HEAD_CHUNK_ROWS``, and each chunk's backward runs right away in the forward (the loss is the last
    op, so its gradient is known up to the upstream scalar g): the xent kernel turns the chunk's logits
    into dlogits in place, dh = dlogits W and dW += dlogits^T h (fp32) are computed, and the chunk's
    logits buffer is reused. ``backward`` only scales by g: dh * g, arena dW += g * dW, db += g * db.
    Peak head memory drops from B*n*V/2 bf16 logits (1.6 GB at B48) to one chunk."""

    @staticmethod
    def forward(ctx, h, w, b, labels, text_seq_len, Vt, img_w):
        if _head_asm_ok(h, w, b, ctx, text_seq_len, Vt):
            return _SplitXent._forward_asm(ctx, h, w, b, labels, text_seq_len, Vt, img_w)
        B, n, d = h.shape
        wb, bb = bf16_weight(w), bf16_weight(b)
        den = 1.0 + img_w
        segs = ((h[:, :text_seq_len], labels[:, :text_seq_len], 0, Vt, 1.0),
                (h[:, text_seq_len:], labels[:, text_seq_len:] - Vt, Vt, w.shape[0], img_w))
        eager = any(ctx.needs_input_grad[:3])  # the backward will be asked for: do its work now
        dh = torch.empty(B, n, d, dtype=torch.bfloat16, device=h.device)
        dW = torch.zeros(w.shape, dtype=torch.float32, device=h.device)
        db = torch.zeros(b.shape, dtype=torch.float32, device=h.device)
        loss = torch.zeros((), dtype=torch.float32, device=h.device)
        col0 = 0
        for hs, ls, v0, v1, wt in segs:
            rows = hs.shape[1]
            hs2 = hs.reshape(-1, d).contiguous()
            ls2 = ls.reshape(-1).contiguous()
            N = hs2.shape[0]
            gscale = wt / (den * N)
            dh_seg = dh[:, col0:col0 + rows].view(-1, d) if dh[:, col0:col0 + rows].is_contiguous() else None
            dh_parts = []
            for r0 in range(0, N, HEAD_CHUNK_ROWS):
                r1 = min(N, r0 + HEAD_CHUNK_ROWS)
                hc = hs2[r0:r1]
                logit = torch.addmm(bb[v0:v1], hc, wb[v0:v1].t())
                if eager and v1 - v0 <= XENT_COLSUM_MAXV:
                    # logit -> dL/dlogits in place, their column sums -> db (the bias gradient)
                    lc = C().xent_colsum_(logit, ls2[r0:r1], gscale, db[v0:v1])
                elif eager:  # vocabulary split wider than the kernel's LDS accumulator
                    lc = C().xent_fwd_bwd_(logit, ls2[r0:r1], gscale)
                    db[v0:v1] += logit.float().sum(0)
                else:
                    lc = C().xent_fwd_bwd_(logit, ls2[r0:r1], gscale)
                loss = loss + lc.sum() * gscale
                if eager:
                    part = torch.mm(logit, wb[v0:v1])
                    if dh_seg is not None:
                        dh_seg[r0:r1].copy_(part)
                    else:
                        dh_parts.append(part)
                    torch.addmm(dW[v0:v1], logit.t(), hc, out_dtype=torch.float32, out=dW[v0:v1])
                del logit
            if eager and dh_seg is None:
                dh[:, col0:col0 + rows] = torch.cat(dh_parts).view(B, rows, d)
            col0 += rows
        ctx.save_for_backward(dh, dW, db)
        ctx.params = (w, b)
        ctx.segs = None
        return loss

    @staticmethod
    def _forward_asm(ctx, h, w, b, labels, text_seq_len, Vt, img_w):
        """The same chunked forward + eager backward with all three head products on the assembly GEMMs:
        logits = h W_s^T + b_s (nt_bias), dh = dlogits W_s (nt_plain against a cached transposed copy,
        K = the split's width), dW_s += dlogits^T h (tn_wgrad, fp32). Each vocabulary split is padded to a
        multiple of 256 columns (the text split: 32356 -> 32512) with zero weight rows and a bias of -3e4:
        a padded logit is -3e4, its probability exp(-3e4 - max) is exactly 0 in fp32, so its dlogit is 0
        and it adds nothing to dh, dW or db; the padded rows of dW / db are dropped in ``backward``."""
        B, n, d = h.shape
        den = 1.0 + img_w
        V = w.shape[0]
        splits = ((h[:, :text_seq_len], labels[:, :text_seq_len], 0, Vt, 1.0),
                  (h[:, text_seq_len:], labels[:, text_seq_len:] - Vt, Vt, V, img_w))
        pads = [-(-(v1 - v0) // 256) * 256 for _, _, v0, v1, _ in splits]
        dh = torch.empty(B, n, d, dtype=torch.bfloat16, device=h.device)
        dW = torch.zeros(sum(pads), d, dtype=torch.float32, device=h.device)
        db = torch.zeros(sum(pads), dtype=torch.float32, device=h.device)
        loss = torch.zeros((), dtype=torch.float32, device=h.device)
        col0, off, segs = 0, 0, []
        for (hs, ls, v0, v1, wt), Vp in zip(splits, pads):
            ws, bs, wst = _head_split_weights(w, b, v0, v1, Vp)
            rows = hs.shape[1]
            hs2 = hs.reshape(-1, d).contiguous()
            ls2 = ls.reshape(-1).contiguous()
            N = hs2.shape[0]
            gscale = wt / (den * N)
            dW_s, db_s = dW[off:off + Vp], db[off:off + Vp]
            sw = asm_wgrad_splits(min(N, HEAD_CHUNK_ROWS), Vp, d)
            dh_parts = []
            for r0 in range(0, N, HEAD_CHUNK_ROWS):
                r1 = min(N, r0 + HEAD_CHUNK_ROWS)
                hc = hs2[r0:r1]
                logit = C().asm_gemm(hc, ws, bs, None)
                lc = C().xent_colsum_(logit, ls2[r0:r1], gscale, db_s)  # logit -> dL/dlogits in place
                loss = loss + lc.sum() * gscale
                dh_parts.append(C().asm_gemm(logit, wst, None, None))
                s = sw if (r1 - r0) == min(N, HEAD_CHUNK_ROWS) else asm_wgrad_splits(r1 - r0, Vp, d)
                C().asm_wgrad_(dW_s, logit, hc, max(s, 1), True)
                del logit
            if dh_parts:
                dh[:, col0:col0 + rows] = (dh_parts[0] if len(dh_parts) == 1 else torch.cat(dh_parts)).view(B, rows, d)
            segs.append((v0, v1, off))
            col0 += rows
            off += Vp
        _count("asm_head")
        ctx.save_for_backward(dh, dW, db)
        ctx.params = (w, b)
        ctx.segs = segs
        return loss

    @staticmethod
    def backward(ctx, gl):
        dh, dW, db = ctx.saved_tensors
        g = gl.float()
        w, b = ctx.params
        gw, gb = grad_sink(w, ctx.needs_input_grad[1]), grad_sink(b, ctx.needs_input_grad[2])
        dh = (dh * g.to(dh.dtype)) if g.numel() else dh
        segs = ctx.segs if ctx.segs is not None else ((0, w.shape[0], 0),)  # padded assembly-path splits
        if gw is not None and gb is not None:  # accumulate into the arena, no host read of g
            for v0, v1, off in segs:
                gw.view(w.shape)[v0:v1].addcmul_(dW[off:off + v1 - v0], g)
                gb.view(b.shape)[v0:v1].addcmul_(db[off:off + v1 - v0], g)
            return dh, None, None, None, None, None, None
        if ctx.segs is not None:
            dW = torch.cat([dW[off:off + v1 - v0] for v0, v1, off in segs])
            db = torch.cat([db[off:off + v1 - v0] for v0, v1, off in segs])
        return dh, dW * g, db * g, None, None, None, None


def _head_asm_ok(h, w, b, ctx, text_seq_len: int, Vt: int) -> bool:
    """The assembly head path: eager (the gradient is wanted), operands on the GPU, d a multiple of 256 (>= 1024), row counts that
    tile (B * text_len and B * image_len multiples of 256) and padded vocabulary splits the fused CE kernel's
    LDS column sums hold; anything else takes the hipBLASLt path."""
    if not (ASM_GEMM and h.is_cuda and all(ctx.needs_input_grad[:3]) and h.dim() == 3 and h.shape[-1] % 256 == 0
            and h.shape[-1] >= 1024
            and HEAD_CHUNK_ROWS % 256 == 0 and w.dim() == 2 and w.shape[1] == h.shape[-1] and b is not None):
        return False
    B, n = h.shape[0], h.shape[1]
    pads = [-(-v // 256) * 256 for v in (Vt, w.shape[0] - Vt)]
    return (B * text_seq_len) % 256 == 0 and (B * (n - text_seq_len)) % 256 == 0 and max(pads) <= XENT_COLSUM_MAXV


def _head_split_weights(w, b, v0: int, v1: int, Vp: int):
    """(W_s padded to Vp rows bf16, b_s padded with -3e4 fp32, W_s^T padded (d, Vp) bf16): the weight copies are
    cached per forward (keyed on W's version), the bias slice is refreshed on every call (a frozen W with a
    trained bias never reads a stale bias)."""
    def make():
        ws = torch.zeros(Vp, w.shape[1], dtype=torch.bfloat16, device=w.device)
        ws[:v1 - v0] = w.detach()[v0:v1]
        bs = torch.full((Vp,), -3.0e4, dtype=torch.float32, device=w.device)
        return ws, bs, ws.t().contiguous()
    ws, bs, wst = _cached(("head", id(w), v0, v1), w, make)
    bs[:v1 - v0].copy_(b.detach()[v0:v1])
    return ws, bs, wst


# rows of one head chunk (logits of 4096 text rows: 265 MB bf16, image rows: 67 MB)
# rows per head chunk: 16384 measured 0.9 % faster per bench24 step than 4096 (6 of 6 same-box pairs,
# profiles/r2_s4_head_chunk_ab.txt) for ~0.55 GB more peak memory (B48: the 12288 text rows form one 0.8 GB
# logits chunk, the image rows three of 0.27 GB; the full 1.6 GB never exists)
HEAD_CHUNK_ROWS = int(os.environ.get("DALLE_AMD_HEAD_CHUNK_ROWS", "16384"))
# widest vocabulary split xent_colsum_ holds in LDS (csrc/kernels/xent.hip XENT_MAXV); wider splits sum in PyTorch
XENT_COLSUM_MAXV = 35000


def logits_loss(out, norm_w, norm_b, weight, bias, labels, text_seq_len: int, num_text_tokens: int, loss_img_weight: float):
    h = _LNShift.apply(out.float() if out.dtype != torch.float32 else out, norm_w, norm_b, 0, 1, False)
    return _SplitXent.apply(h, weight, bias, labels, text_seq_len, num_text_tokens, float(loss_img_weight))


def nonfinite_flag(x: torch.Tensor) -> torch.Tensor:
    return C().nonfinite(x.contiguous())


def zero_if_nonfinite_(x: torch.Tensor) -> torch.Tensor:
    assert x.is_contiguous() and x.dtype == torch.float32
    return C().zero_if_nonfinite_(x)
