"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op (MI355X only)."""
import pytest
import torch
import torch.nn.functional as F

from dalle_amd.models.patterns import AttnGeometry, PATTERN_IDS
from dalle_amd.models.rotary import rotary_tables
from dalle_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

GEOMS = [(65, 16), (257, 32)]  # (text_len, image side): tiny and the reference geometry


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("T,S", GEOMS)
@pytest.mark.parametrize("D", [256, 1024])
@pytest.mark.parametrize("shift", [True, False])
def test_layernorm_shift(cuda, T, S, D, shift):
    from dalle_amd.ops import hip_ops

    torch.manual_seed(0)
    B, n = 2, T + S * S - 1
    x = torch.randn(B, n, D, device=cuda, requires_grad=True)
    w = (1 + 0.1 * torch.randn(D, device=cuda)).requires_grad_(True)
    b = (0.1 * torch.randn(D, device=cuda)).requires_grad_(True)
    y = hip_ops.layernorm_shift(x, w, b, T, S, shift)
    xr, wr, br = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    yr = ref.layernorm_shift(xr, wr, br, T, S, shift)
    assert y.dtype == torch.bfloat16
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g.to(torch.bfloat16))
    yr.backward(g.to(torch.bfloat16).float())
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2


@pytest.mark.parametrize("T,S", GEOMS)
@pytest.mark.parametrize("attn_type", ["axial_row", "axial_col", "conv_like", "full"])
def test_sparse_attention(cuda, T, S, attn_type):
    from dalle_amd.ops import hip_ops

    torch.manual_seed(1)
    B, H, Dh = 2, 2, 64
    n = T + S * S - 1
    geom = AttnGeometry(T, S, 5)
    qkv = (torch.randn(B, n, 3 * H * Dh, device=cuda) * 1.5).to(torch.bfloat16).requires_grad_(True)
    out = hip_ops.attention_core(qkv, H, geom, attn_type)
    cos, sin = rotary_tables(T, S, Dh, device=cuda)
    qr_in = qkv.detach().float().requires_grad_(True)
    q, k, v = ref.qkv_rotary(qr_in, H, cos, sin)
    out_ref = ref.sparse_attention_core(q, k, v, geom, attn_type)
    assert torch.isfinite(out.float()).all()
    assert _rel(out, out_ref) < 2e-2, attn_type
    g = torch.randn_like(out_ref)
    out.backward(g.to(torch.bfloat16))
    out_ref.backward(g.to(torch.bfloat16).float())
    assert _rel(qkv.grad, qr_in.grad) < 3e-2, attn_type


def test_geglu(cuda):
    from dalle_amd.ops import hip_ops

    torch.manual_seed(2)
    h = torch.randn(300, 2 * 512, device=cuda).to(torch.bfloat16).requires_grad_(True)
    y = hip_ops._GEGLU.apply(h)
    hr = h.detach().float().requires_grad_(True)
    yr = ref.geglu(hr)
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    assert _rel(h.grad, hr.grad) < 1e-2


def test_scale_residual(cuda):
    from dalle_amd.ops import hip_ops

    torch.manual_seed(3)
    x = torch.randn(4, 100, 256, device=cuda, requires_grad=True)
    y = torch.randn(4, 100, 256, device=cuda).to(torch.bfloat16).requires_grad_(True)
    s = torch.rand(1, 1, 256, device=cuda, requires_grad=True)
    o = hip_ops.scale_residual(x, y, s)
    xr, yr, sr = x.detach().clone().requires_grad_(True), y.detach().float().requires_grad_(True), s.detach().clone().requires_grad_(True)
    orf = xr + yr * sr
    assert _rel(o, orf) < 1e-5
    g = torch.randn_like(orf)
    o.backward(g)
    orf.backward(g)
    assert _rel(x.grad, xr.grad) < 1e-6
    assert _rel(y.grad, yr.grad) < 1e-2
    assert _rel(s.grad, sr.grad) < 1e-4


@pytest.mark.parametrize("V", [8192, 32356, 1000])
def test_xent(cuda, V):
    from dalle_amd.ops import hip_ops

    torch.manual_seed(4)
    R = 37
    logits = (torch.randn(R, V, device=cuda) * 3).to(torch.bfloat16)
    labels = torch.randint(0, V, (R,), device=cuda)
    ref_logits = logits.float().requires_grad_(True)
    loss_ref = F.cross_entropy(ref_logits, labels, reduction="none")
    loss_ref.sum().backward()
    buf = logits.clone()
    loss = hip_ops.C().xent_fwd_bwd_(buf, labels, 1.0)
    assert torch.allclose(loss, loss_ref, atol=2e-3, rtol=1e-3)
    assert _rel(buf, ref_logits.grad) < 1e-2


@pytest.mark.parametrize("chunk", [4096, 100])
def test_split_logits_loss(cuda, chunk, monkeypatch):
    """K12 chunked head (several chunks + a ragged last one when chunk=100) with an upstream gradient
    scale of 3 (the eager in-forward backward must scale by it)."""
    from dalle_amd.ops import hip_ops

    monkeypatch.setattr(hip_ops, "HEAD_CHUNK_ROWS", chunk)
    torch.manual_seed(5)
    B, tsl, n_img, d, Vt, Vi = 2, 64, 256, 256, 1064, 512
    n = tsl + n_img
    out = torch.randn(B, n, d, device=cuda, requires_grad=True)
    nw = torch.ones(d, device=cuda, requires_grad=True)
    nb = torch.zeros(d, device=cuda, requires_grad=True)
    W = (torch.randn(Vt + Vi, d, device=cuda) * 0.05).requires_grad_(True)
    bias = torch.zeros(Vt + Vi, device=cuda, requires_grad=True)
    labels = torch.cat([torch.randint(0, Vt, (B, tsl)), torch.randint(Vt, Vt + Vi, (B, n_img))], 1).to(cuda)
    hip_ops.begin_forward()
    loss = hip_ops.logits_loss(out, nw, nb, W, bias, labels, tsl, Vt, 7.0)
    (loss * 3.0).backward()
    o2, W2, b2 = (t.detach().clone().requires_grad_(True) for t in (out, W, bias))
    h = F.layer_norm(o2, (d,))
    loss_r = ref.split_logits_loss(h, W2, b2, labels, tsl, Vt, 7.0)
    (loss_r * 3.0).backward()
    assert abs(loss.item() - loss_r.item()) < 1e-2
    assert _rel(out.grad, o2.grad) < 3e-2
    assert _rel(W.grad, W2.grad) < 3e-2
    assert _rel(bias.grad, b2.grad) < 3e-2


@pytest.mark.parametrize("chunk", [16384, 256])
def test_split_logits_loss_asm_head(cuda, chunk, monkeypatch):
    """K12 on the assembly GEMMs (d = 1024): logits / dh / dW through nt_bias / nt_plain / tn_wgrad, the text
    split padded 1064 -> 1280 columns (zero rows, bias -3e4), one or several chunks; checked against fp32."""
    from dalle_amd.ops import hip_ops

    monkeypatch.setattr(hip_ops, "HEAD_CHUNK_ROWS", chunk)
    torch.manual_seed(6)
    B, tsl, n_img, d, Vt, Vi = 2, 256, 512, 1024, 1064, 512
    n = tsl + n_img
    out = torch.randn(B, n, d, device=cuda, requires_grad=True)
    nw = torch.ones(d, device=cuda, requires_grad=True)
    nb = torch.zeros(d, device=cuda, requires_grad=True)
    W = (torch.randn(Vt + Vi, d, device=cuda) * 0.03).requires_grad_(True)
    bias = (torch.randn(Vt + Vi, device=cuda) * 0.1).requires_grad_(True)
    labels = torch.cat([torch.randint(0, Vt, (B, tsl)), torch.randint(Vt, Vt + Vi, (B, n_img))], 1).to(cuda)
    hip_ops.begin_forward()
    before = hip_ops.PATH_COUNTS.get("asm_head", 0)
    loss = hip_ops.logits_loss(out, nw, nb, W, bias, labels, tsl, Vt, 7.0)
    (loss * 3.0).backward()
    assert hip_ops.PATH_COUNTS.get("asm_head", 0) == before + 1, "the assembly head path did not run"
    o2, W2, b2 = (t.detach().clone().requires_grad_(True) for t in (out, W, bias))
    h = F.layer_norm(o2, (d,))
    loss_r = ref.split_logits_loss(h, W2, b2, labels, tsl, Vt, 7.0)
    (loss_r * 3.0).backward()
    assert abs(loss.item() - loss_r.item()) < 1e-2
    assert _rel(out.grad, o2.grad) < 3e-2
    assert _rel(W.grad, W2.grad) < 3e-2
    assert _rel(bias.grad, b2.grad) < 3e-2


def test_asm_head_sees_bias_updates(cuda):
    """The padded head weights are cached per forward; a bias changed in place (W untouched, no begin_forward)
    must still reach the logits: the loss matches the fp32 reference with the NEW bias."""
    from dalle_amd.ops import hip_ops

    torch.manual_seed(7)
    B, tsl, n_img, d, Vt, Vi = 1, 256, 256, 1024, 700, 512
    n = tsl + n_img
    out = torch.randn(B, n, d, device=cuda, requires_grad=True)
    nw = torch.ones(d, device=cuda, requires_grad=True)
    nb = torch.zeros(d, device=cuda, requires_grad=True)
    W = (torch.randn(Vt + Vi, d, device=cuda) * 0.03).requires_grad_(True)
    bias = torch.zeros(Vt + Vi, device=cuda, requires_grad=True)
    labels = torch.cat([torch.randint(0, Vt, (B, tsl)), torch.randint(Vt, Vt + Vi, (B, n_img))], 1).to(cuda)
    hip_ops.begin_forward()
    hip_ops.logits_loss(out, nw, nb, W, bias, labels, tsl, Vt, 7.0).backward()
    with torch.no_grad():
        bias.add_(torch.randn_like(bias))
    loss = hip_ops.logits_loss(out, nw, nb, W, bias, labels, tsl, Vt, 7.0)
    h = F.layer_norm(out.detach(), (d,))
    loss_r = ref.split_logits_loss(h, W.detach(), bias.detach(), labels, tsl, Vt, 7.0)
    assert abs(loss.item() - loss_r.item()) < 1e-2


def test_nonfinite(cuda):
    from dalle_amd.ops import hip_ops

    x = torch.randn(100003, device=cuda)
    assert int(hip_ops.nonfinite_flag(x)) == 0
    x[77777] = float("nan")
    assert int(hip_ops.nonfinite_flag(x)) == 1


@pytest.mark.parametrize("n", [1000, 300_007, 5_000_000])
def test_uniform8bit_quantization_kernel(cuda, n):
    """HIP 8-bit averaging compression vs a float64 NumPy-style reference of the same algorithm."""
    from dalle_amd.parallel.compression import Uniform8BitQuantization

    torch.manual_seed(0)
    x = (torch.randn(n, device=cuda) * 0.3 + 0.05).float()
    comp = Uniform8BitQuantization()
    c = comp.compress(x)
    xd = x.double()
    mean = xd.mean()
    std = ((xd - mean) ** 2).sum().div(max(n - 1, 1)).sqrt()
    scale = 6 * std / 256
    qref = torch.clamp(torch.round((xd - mean) / scale) + 128, 0, 255).long()
    mismatch = (c["idx"].long() != qref).float().mean().item()
    assert mismatch < 1e-3  # only exact rounding ties at bin edges may differ
    sums = torch.zeros(256, dtype=torch.float64, device=cuda).scatter_add_(0, qref, xd)
    cnts = torch.zeros(256, dtype=torch.float64, device=cuda).scatter_add_(0, qref, torch.ones_like(xd))
    cb_ref = (sums / cnts.clamp_min(1)).float()
    used = cnts > 0
    assert torch.allclose(c["codebook"][used], cb_ref[used], rtol=1e-3, atol=1e-5)
    # deterministic: a second run is bit-identical
    c2 = comp.compress(x)
    assert torch.equal(c["idx"], c2["idx"]) and torch.equal(c["codebook"], c2["codebook"])
    back = comp.extract(c, n)
    assert ((back - x).norm() / x.norm()).item() < 0.05


# ---- randomised geometries (hypothesis): ragged text lengths, both image grids, every pattern ----
from hypothesis import given, settings, strategies as hst  # noqa: E402


@settings(max_examples=10, deadline=None)
@given(T=hst.integers(1, 300), S=hst.sampled_from([16, 32]), B=hst.integers(1, 2), H=hst.integers(1, 3),
       attn_type=hst.sampled_from(["axial_row", "axial_col", "conv_like", "full"]), seed=hst.integers(0, 999))
def test_sparse_attention_random_geometry(cuda, T, S, B, H, attn_type, seed):
    from dalle_amd.ops import hip_ops
    dev = cuda
    torch.manual_seed(seed)
    n = T + S * S - 1
    geom = AttnGeometry(T, S, 5)
    qkv = (torch.randn(B, n, 3 * H * 64, device=dev) * 1.5).to(torch.bfloat16).requires_grad_(True)
    out = hip_ops.attention_core(qkv, H, geom, attn_type)
    cos, sin = rotary_tables(T, S, 64, device=dev)
    qr_in = qkv.detach().float().requires_grad_(True)
    q, k, v = ref.qkv_rotary(qr_in, H, cos, sin)
    out_ref = ref.sparse_attention_core(q, k, v, geom, attn_type)
    assert _rel(out, out_ref) < 2e-2, (T, S, attn_type)
    g = torch.randn_like(out_ref)
    out.backward(g.to(torch.bfloat16))
    out_ref.backward(g.to(torch.bfloat16).float())
    assert _rel(qkv.grad, qr_in.grad) < 3e-2, (T, S, attn_type)


@settings(max_examples=10, deadline=None)
@given(T=hst.integers(1, 300), S=hst.sampled_from([16, 32]), D=hst.sampled_from([256, 1024]), shift=hst.booleans(),
       seed=hst.integers(0, 999))
def test_layernorm_shift_random_geometry(cuda, T, S, D, shift, seed):
    from dalle_amd.ops import hip_ops
    dev = cuda
    torch.manual_seed(seed)
    n = T + S * S - 1
    x = torch.randn(2, n, D, device=dev, requires_grad=True)
    w = (1 + 0.1 * torch.randn(D, device=dev)).requires_grad_(True)
    b = (0.1 * torch.randn(D, device=dev)).requires_grad_(True)
    y = hip_ops.layernorm_shift(x, w, b, T, S, shift)
    xr, wr, br = (t.detach().clone().requires_grad_(True) for t in (x, w, b))
    yr = ref.layernorm_shift(xr, wr, br, T, S, shift)
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    assert _rel(x.grad, xr.grad) < 2e-2 and _rel(w.grad, wr.grad) < 2e-2 and _rel(b.grad, br.grad) < 2e-2


@pytest.mark.parametrize("attn_type", ["axial_row", "axial_col", "conv_like", "full"])
def test_fused_rotary_backward_matches_separate_pass(cuda, attn_type):
    """attn_bwd_rope (rotary backward in the attention-backward epilogues) == attn_bwd + rope_bwd."""
    from dalle_amd.models.patterns import PATTERN_IDS
    from dalle_amd.ops import hip_ops

    C = hip_ops.C()
    torch.manual_seed(3)
    T, S, B, H = 257, 32, 2, 3
    n = T + S * S - 1
    geom = AttnGeometry(T, S, 5)
    qkv = (torch.randn(B, n, 3 * H * 64, device=cuda)).to(torch.bfloat16)
    g = torch.randn(B, n, H * 64, device=cuda).to(torch.bfloat16)
    x = qkv.clone().requires_grad_(True)
    hip_ops.attention_core(x, H, geom, attn_type).backward(g)
    cos, sin = rotary_tables(T, S, 64, device=cuda)
    col, pat = attn_type == "axial_col", PATTERN_IDS[attn_type]
    q, k, v = C.rope_fwd(qkv, cos, sin, T, S, H, col, 0.125)
    out, lse = C.attn_fwd(q, k, v, B, T, S, n, geom.kernel_size, H, pat)
    dq, dk, dv = C.attn_bwd(q, k, v, out, g, lse, B, T, S, n, geom.kernel_size, H, pat)
    grads = [x.grad.float(), C.rope_bwd(dq, dk, dv, cos, sin, B, T, S, H, n, col, 0.125).float().view_as(x.grad)]
    # one bf16 rounding (fused) vs two (separate pass)
    assert _rel(grads[0], grads[1]) < 8e-3, attn_type


@pytest.mark.parametrize("T,B,H", [(257, 2, 3), (260, 1, 2), (65, 2, 2), (1, 1, 1), (256, 1, 2), (261, 1, 1)])
@pytest.mark.parametrize("attn_type", ["axial_row", "axial_col"])
def test_fused_one_workgroup_backward(cuda, attn_type, T, B, H, monkeypatch):
    """The one-workgroup-per-head axial backward (S = 32: dQ, dK, dV from one S / dP per tile pair, the 9th
    text tile's real keys accumulated in LDS) == the two-kernel backward (DALLE_AMD_ATTN_FUSED_BWD=0) to bf16
    resolution, and the fp32 reference. The fused kernel computes the rotary angles in-kernel (frequencies
    of rotary.rotary_freq_split), the two-kernel form reads the tables: this also pins the two against each other."""
    from dalle_amd.models.patterns import PATTERN_IDS
    from dalle_amd.ops import hip_ops

    C = hip_ops.C()
    torch.manual_seed(11 + T)
    S = 32
    n = T + S * S - 1
    geom = AttnGeometry(T, S, 5)
    qkv = torch.randn(B, n, 3 * H * 64, device=cuda).to(torch.bfloat16)
    g = torch.randn(B, n, H * 64, device=cuda).to(torch.bfloat16)
    cos, sin = rotary_tables(T, S, 64, device=cuda)
    col, pat = attn_type == "axial_col", PATTERN_IDS[attn_type]
    q, k, v = C.rope_fwd(qkv, cos, sin, T, S, H, col, 0.125)
    out, lse = C.attn_fwd(q, k, v, B, T, S, n, geom.kernel_size, H, pat)
    rf = hip_ops._rot_freqs(q.device)
    monkeypatch.setenv("DALLE_AMD_ATTN_FUSED_BWD", "1")
    fused = C.attn_bwd_rope(q, k, v, out, g, lse, cos, sin, B, T, S, n, geom.kernel_size, H, pat, 0.125, *rf).float()
    monkeypatch.setenv("DALLE_AMD_ATTN_FUSED_BWD", "0")
    two = C.attn_bwd_rope(q, k, v, out, g, lse, cos, sin, B, T, S, n, geom.kernel_size, H, pat, 0.125, *rf).float()
    torch.cuda.synchronize()
    assert torch.isfinite(fused).all()
    assert _rel(fused, two) < 8e-3, (attn_type, T)
    for part in range(3):   # q, k and v gradients each (a missing store would hide in the total)
        sl = slice(part * H * 64, (part + 1) * H * 64)
        assert _rel(fused[..., sl], two[..., sl]) < 8e-3, (attn_type, T, part)
    xr = qkv.float().requires_grad_(True)
    qr, kr, vr = ref.qkv_rotary(xr, H, cos, sin)
    ref.sparse_attention_core(qr, kr, vr, geom, attn_type).backward(g.float())
    assert _rel(fused.view_as(xr.grad), xr.grad) < 3e-2, attn_type


@pytest.mark.parametrize("S", [16, 32])
@pytest.mark.parametrize("attn_type", ["axial_row", "axial_col"])
def test_axial_local_dkdv_fused_into_dq_kernel(cuda, attn_type, S, monkeypatch):
    """Axial patterns: the image keys' dK / dV computed inside the dQ kernel (the rotary-fused backward the
    model runs) must match the separate key-centric kernel's (attn_bwd + rope_bwd) to bf16 resolution, and the
    fp32 reference."""
    from dalle_amd.models.patterns import PATTERN_IDS
    from dalle_amd.ops import hip_ops

    C = hip_ops.C()
    monkeypatch.setenv("DALLE_AMD_ATTN_FUSED_BWD", "0")   # the two-kernel form (the fused one: test above)
    torch.manual_seed(5)
    T, B, H = 65, 2, 2
    n = T + S * S - 1
    geom = AttnGeometry(T, S, 5)
    qkv = torch.randn(B, n, 3 * H * 64, device=cuda).to(torch.bfloat16)
    g = torch.randn(B, n, H * 64, device=cuda).to(torch.bfloat16)
    x = qkv.clone().requires_grad_(True)
    hip_ops.attention_core(x, H, geom, attn_type).backward(g)
    fused = x.grad.float()
    cos, sin = rotary_tables(T, S, 64, device=cuda)
    col = attn_type == "axial_col"
    pat = PATTERN_IDS[attn_type]
    q, k, v = C.rope_fwd(qkv, cos, sin, T, S, H, col, 0.125)
    out, lse = C.attn_fwd(q, k, v, B, T, S, n, geom.kernel_size, H, pat)
    dq, dk, dv = C.attn_bwd(q, k, v, out, g, lse, B, T, S, n, geom.kernel_size, H, pat)
    sep = C.rope_bwd(dq, dk, dv, cos, sin, B, T, S, H, n, col, 0.125).float().view_as(fused)
    torch.cuda.synchronize()
    assert torch.isfinite(fused).all()
    # the separate chain rounds dQ / dK / dV to bf16 before its rotary backward; the fused epilogues rotate
    # the fp32 values: equal to bf16 resolution
    assert _rel(fused, sep) < 8e-3, attn_type
    xr = qkv.float().requires_grad_(True)
    q, k, v = ref.qkv_rotary(xr, H, cos, sin)
    ref.sparse_attention_core(q, k, v, geom, attn_type).backward(g.float())
    assert _rel(fused, xr.grad) < 3e-2, attn_type


def test_segmented_uniform8bit_matches_per_part(cuda):
    """One segmented launch (one workgroup per part, csrc/kernels/quant.hip) == the per-part quantiser
    (same indices up to rounding ties, same per-part codebooks), and the segmented dequantiser puts every
    part back at its own offset (accumulating or not)."""
    from dalle_amd.parallel.averaging import _seg_compress, _seg_dequant
    from dalle_amd.parallel.compression import Uniform8BitQuantization

    torch.manual_seed(0)
    x = torch.randn(700_000, device=cuda)
    x[200_000:400_000] *= 1e-3  # parts of very different scale
    parts = [(0, 131072), (131072, 68928), (200_000, 131072), (331_072, 68928), (450_000, 5), (500_000, 200_000)]
    x_off = torch.tensor([o for o, _ in parts], dtype=torch.int64, device=cuda)
    lens = torch.tensor([n for _, n in parts], dtype=torch.int32, device=cuda)
    q_off = torch.tensor([0] + list(torch.tensor([n for _, n in parts]).cumsum(0)[:-1].tolist()), dtype=torch.int64,
                         device=cuda)
    total = sum(n for _, n in parts)
    q = torch.empty(total, dtype=torch.uint8, device=cuda)
    cb = torch.empty(len(parts) * 256, dtype=torch.float32, device=cuda)
    _seg_compress(x, x_off, q_off, lens, q, cb, 700_000, total)
    quant = Uniform8BitQuantization()
    for i, ((o, n), qo) in enumerate(zip(parts, q_off.tolist())):
        ref = quant.compress(x[o:o + n].contiguous())
        mism = (q[qo:qo + n] != ref["idx"]).float().mean().item()
        assert mism < 2e-3, (i, mism)
        used = torch.bincount(ref["idx"].long(), minlength=256) > 0
        assert torch.allclose(cb[i * 256:(i + 1) * 256][used], ref["codebook"][used], rtol=1e-3, atol=1e-7), i
    out = torch.zeros(700_000, device=cuda)
    _seg_dequant(q, q_off, cb, x_off, lens, out, total, 700_000, accumulate=False)
    _seg_dequant(q, q_off, cb, x_off, lens, out, total, 700_000, accumulate=True)
    for o, n in parts:
        rel = ((out[o:o + n] / 2 - x[o:o + n]).norm() / x[o:o + n].norm()).item()
        assert rel < 0.05, (o, rel)
    assert out[450_005:500_000].abs().max().item() == 0.0  # outside every part: untouched


def test_debug_sync_mode_wraps_every_native_op(cuda, monkeypatch):
    """DALLE_AMD_DEBUG_SYNC=1: the native ops run through a synchronising proxy."""
    from dalle_amd.ops import hip_ops

    monkeypatch.setenv("DALLE_AMD_DEBUG_SYNC", "1")
    monkeypatch.setattr(hip_ops, "_C", None)
    try:
        C = hip_ops.C()
        assert isinstance(C, hip_ops._SyncedExtension)
        x = torch.randn(4096, device=cuda)
        assert int(C.nonfinite(x).item()) == 0
    finally:
        monkeypatch.setattr(hip_ops, "_C", None)


@pytest.mark.parametrize("B,T,I,d", [(3, 64, 256, 256), (2, 256, 1024, 1024)])
def test_embedding_kernel(cuda, B, T, I, d):
    """K1+K2: pad remap + BOS + tied-table gather (fp32 out) and the deterministic segmented backward into
    the arena grad vs index_add in float64; two backward runs are bitwise identical."""
    from dalle_amd.ops import hip_ops
    from dalle_amd.optim import FlatArena

    torch.manual_seed(0)
    Vtext0, n_img = 1000, 512
    Vt = Vtext0 + T
    table = torch.nn.Parameter(torch.randn(Vt + n_img, d, device=cuda))
    arena = FlatArena([table], device=cuda)
    text = torch.randint(1, 300, (B, T), device=cuda)
    text[:, T // 2:] = 1          # eos padding: one long run of a single id
    text[0, 3] = 0                # a 0 -> unique pad id of position 3
    image = torch.randint(0, n_img, (B, I), device=cuda)
    out = hip_ops.embed_tokens(text, image, table, Vtext0, Vt)
    ids = torch.cat([torch.zeros(B, 1, dtype=torch.long, device=cuda),
                     torch.where(text == 0, torch.arange(T, device=cuda) + Vtext0, text), image[:, :-1] + Vt], 1)
    assert out.shape == (B, T + I, d) and out.dtype == torch.float32
    assert torch.equal(out, table.detach()[ids])
    g = torch.randn_like(out)
    grads = []
    for _ in range(2):
        arena.zero_grad()
        out = hip_ops.embed_tokens(text, image, table, Vtext0, Vt)
        out.backward(g)
        grads.append(arena.grad.clone())
    assert torch.equal(grads[0], grads[1])
    ref = torch.zeros(table.shape, dtype=torch.float64, device=cuda).index_add_(0, ids.reshape(-1), g.reshape(-1, d).double())
    assert torch.allclose(table.grad.double(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("shape", [(3072, 1024), (1024, 4096), (8192, 1024), (37, 70), (1, 33)])
def test_transpose_cast_bf16_bitwise(cuda, shape):
    """fp32 W -> bf16 W^T in one tiled pass (the input-gradient operand copy) == cast then transpose."""
    from dalle_amd.ops.hip_ops import C

    w = torch.randn(*shape, device=cuda) * 3.0
    got = C().transpose_bf16(w)
    assert torch.equal(got, w.bfloat16().t().contiguous())


@pytest.mark.parametrize("V", [8192, 32356, 1064, 516, 1000])
def test_xent_colsum(cuda, V):
    """Fused CE + in-place dlogits + bias-gradient column sums (register-resident forms up to 32768 columns,
    the LDS-accumulator form beyond) against fp32 PyTorch; the column sums are of the bf16 dlogits the GEMMs
    consume."""
    from dalle_amd.ops import hip_ops

    C = hip_ops.C()
    torch.manual_seed(6)
    R = 2000
    logits = (torch.randn(R, V, device=cuda) * 3).to(torch.bfloat16)
    labels = torch.randint(0, V, (R,), device=cuda)
    ref_logits = logits.float().requires_grad_(True)
    loss_ref = F.cross_entropy(ref_logits, labels, reduction="none")
    (loss_ref.sum() * 0.25).backward()
    buf = logits.clone()
    db = torch.full((V,), 0.5, device=cuda)
    loss = C.xent_colsum_(buf, labels, 0.25, db)
    torch.cuda.synchronize()
    assert torch.allclose(loss, loss_ref, atol=2e-3, rtol=1e-3)
    assert _rel(buf, ref_logits.grad) < 1e-2
    assert torch.allclose(db - 0.5, buf.float().sum(0), atol=1e-4, rtol=1e-4)  # += into the sink
    buf2 = logits.clone()
    db2 = torch.full((V,), 0.5, device=cuda)
    C.xent_colsum_(buf2, labels, 0.25, db2)
    assert torch.equal(buf2, buf) and torch.equal(db2, db)  # deterministic


@pytest.mark.parametrize("R,Cc", [(64, 64), (1280, 1024), (4096, 192)])
def test_transpose_act_bf16(cuda, R, Cc):
    """bf16 activation transpose (the token-contiguous weight-grad input) is a bitwise copy of x.t()."""
    from dalle_amd.ops.ext import load_extension

    C = load_extension(required=True)
    torch.manual_seed(0)
    x = torch.randn(R, Cc, device=cuda).bfloat16()
    xt = C.transpose_act_bf16(x)
    assert xt.shape == (Cc, R) and xt.is_contiguous()
    assert torch.equal(xt, x.t().contiguous())


@pytest.mark.parametrize("M,N,K", [(81920 // 16, 3072, 1024), (20480, 8192, 1024), (2048, 1024, 4096), (512, 256, 128)])
@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("form", ["xt", "gt", "nt"])
def test_weight_grad_token_contiguous_input(cuda, M, N, K, fused, form):
    """dW = g^T x with x and / or g given as token-contiguous XT copies (split-K over strided views, fp32
    partials + fold) matches the fp32 reference, accumulating into an existing fp32 grad (the arena) or
    returning a fresh one."""
    from dalle_amd.ops import hip_ops

    torch.manual_seed(0)
    g = torch.randn(M, N, device=cuda).bfloat16()
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = torch.nn.Parameter(torch.zeros(N, K, device=cuda))
    base = torch.randn(N, K, device=cuda)
    if fused:
        w.grad = base.clone()
    sx = hip_ops.saved_gemm_input(x, True) if form != "gt" else x
    sg = hip_ops.saved_gemm_input(g, True) if form != "xt" else g
    assert isinstance(sx, hip_ops.XT) == (form != "gt") and sx.shape == (M, K) and sg.shape == (M, N)
    r = hip_ops.weight_grad(w, sg, sx)
    want = g.float().t() @ x.float() + (base if fused else 0)
    got = w.grad if fused else r
    assert (r is None) == fused
    assert _rel(got, want) < 1e-5
    # and the token-major form agrees to fp32 rounding
    if fused:
        w.grad = base.clone()
    r2 = hip_ops.weight_grad(w, g, x)
    got2 = w.grad if fused else r2
    assert _rel(got, got2) < 1e-5


