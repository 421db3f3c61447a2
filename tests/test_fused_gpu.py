"""Fused sublayer autograd nodes, split-K weight grads and grad-arena accumulation vs fp32 PyTorch
references (MI355X only)."""
import pytest
import torch

from dalle_amd.models.patterns import AttnGeometry
from dalle_amd.models.rotary import rotary_tables
from dalle_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _params(shapes, device, scale=0.05):
    out = []
    for s in shapes:
        p = torch.nn.Parameter(scale * torch.randn(*s, device=device))
        out.append(p)
    return out


def _arena_grads(params, seed_val):
    """Pre-existing fp32 grads (as the flat arena provides): the fused path must ADD into them."""
    for p in params:
        p.grad = torch.full_like(p, seed_val)


@pytest.mark.parametrize("attn_type", ["axial_row", "axial_col", "conv_like"])
@pytest.mark.parametrize("arena", [False, True])
def test_attn_sublayer(cuda, attn_type, arena):
    from dalle_amd.ops import hip_ops

    torch.manual_seed(0)
    T, S, D, H = 65, 16, 256, 4
    geom = AttnGeometry(T, S, 5)
    B, n = 2, T + S * S - 1
    x = torch.randn(B, n, D, device=cuda, requires_grad=True)
    ln_w, ln_b, w_qkv, w_out, b_out, scale = _params([(D,), (D,), (3 * D, D), (D, D), (D,), (1, 1, D)], cuda)
    with torch.no_grad():
        ln_w.add_(1.0)
        scale.fill_(0.1).add_(0.02 * torch.randn_like(scale))
    params = [ln_w, ln_b, w_qkv, w_out, b_out, scale]
    if arena:
        _arena_grads(params, 0.5)
    y = hip_ops.attn_sublayer(x, *params, H, geom, attn_type, True)
    # reference: fp32 PyTorch composition of the same op
    xr = x.detach().clone().requires_grad_(True)
    pr = [p.detach().clone().requires_grad_(True) for p in params]
    cos, sin = rotary_tables(T, S, 64, device=cuda)
    h = ref.layernorm_shift(xr, pr[0], pr[1], T, S, True)
    o = ref.attention_block(h, pr[2], pr[3], pr[4], H, geom, attn_type, cos, sin)
    yr = xr + o * pr[5]
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    assert _rel(x.grad, xr.grad) < 3e-2
    for p, q in zip(params, pr):
        got = p.grad - 0.5 if arena else p.grad
        assert _rel(got, q.grad) < 3e-2, (p.shape, _rel(got, q.grad))


@pytest.mark.parametrize("arena", [False, True])
def test_ff_sublayer(cuda, arena):
    from dalle_amd.ops import hip_ops

    torch.manual_seed(0)
    T, S, D = 65, 16, 256
    B, n = 2, T + S * S - 1
    x = torch.randn(B, n, D, device=cuda, requires_grad=True)
    ln_w, ln_b, w1, b1, w2, b2, scale = _params([(D,), (D,), (8 * D, D), (8 * D,), (D, 4 * D), (D,), (1, 1, D)], cuda)
    with torch.no_grad():
        ln_w.add_(1.0)
        scale.fill_(0.1)
    params = [ln_w, ln_b, w1, b1, w2, b2, scale]
    if arena:
        _arena_grads(params, -0.25)
    y = hip_ops.ff_sublayer(x, *params, T, S, True)
    xr = x.detach().clone().requires_grad_(True)
    pr = [p.detach().clone().requires_grad_(True) for p in params]
    h = ref.layernorm_shift(xr, pr[0], pr[1], T, S, True)
    yr = xr + ref.feed_forward(h, pr[2], pr[3], pr[4], pr[5]) * pr[6]
    assert _rel(y, yr) < 1e-2
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    assert _rel(x.grad, xr.grad) < 3e-2
    for p, q in zip(params, pr):
        got = p.grad + 0.25 if arena else p.grad
        assert _rel(got, q.grad) < 3e-2, (p.shape, _rel(got, q.grad))


@pytest.mark.parametrize("N,K", [(1024, 1024), (3072, 1024), (1024, 4096)])
@pytest.mark.parametrize("arena", [False, True])
def test_weight_grad_splitk(cuda, N, K, arena):
    from dalle_amd.ops import hip_ops

    torch.manual_seed(0)
    M = 8192
    assert hip_ops.wgrad_splits(M, N, K) > 1
    g2 = torch.randn(M, N, device=cuda).to(torch.bfloat16)
    x2 = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w = torch.nn.Parameter(torch.zeros(N, K, device=cuda))
    want = g2.float().t() @ x2.float()
    if arena:
        w.grad = torch.ones(N, K, device=cuda)
        assert hip_ops.weight_grad(w, g2, x2) is None
        got = w.grad - 1.0
    else:
        got = hip_ops.weight_grad(w, g2, x2)
    assert got.dtype == torch.float32
    assert _rel(got, want) < 1e-4


def test_splitk_accum(cuda):
    from dalle_amd.ops.hip_ops import C

    part = torch.randn(5, 64, 48, device=cuda)
    acc = torch.randn(64, 48, device=cuda)
    want = acc + part.sum(0)
    C().splitk_accum_(acc, part, True)
    assert torch.allclose(acc, want, atol=1e-5)
    C().splitk_accum_(acc, part, False)
    assert torch.allclose(acc, part.sum(0), atol=1e-5)


@pytest.mark.parametrize("variant", [0, 202, 300, 301, 308, 404])
@pytest.mark.parametrize("M,N,K", [(512, 768, 320), (1024, 256, 1024), (256, 256, 64), (768, 512, 128), (2048, 1024, 192)])
def test_gemm_nt(cuda, variant, M, N, K):
    from dalle_amd.ops.hip_ops import C

    torch.manual_seed(0)
    A = torch.randn(M, K, device=cuda).bfloat16()
    B = torch.randn(N, K, device=cuda).bfloat16()
    bias = torch.randn(N, device=cuda).bfloat16()
    want = A.float() @ B.float().t() + bias.float()
    got = C().gemm_nt(A, B, bias, variant).float()
    assert _rel(got, want) < 1e-2
    got = C().gemm_nt(A, B, None, variant).float()
    assert _rel(got, A.float() @ B.float().t()) < 1e-2
    # the pipelined kernels must agree bitwise with the plain one (same MFMA order per output)
    if variant:
        assert torch.equal(C().gemm_nt(A, B, bias, variant), C().gemm_nt(A, B, bias, 0))


@pytest.mark.parametrize("attn_type", ["axial_row", "axial_col"])
def test_qkv_rope_gemm_matches_unfused(cuda, attn_type):
    from dalle_amd.ops.hip_ops import C, _rope_tables

    torch.manual_seed(0)
    T, S, H, D = 65, 16, 4, 256
    geom = AttnGeometry(T, S, 5)
    n, B = T + S * S - 1, 4  # M = 1280: a multiple of 256
    h = torch.randn(B * n, D, device=cuda).bfloat16()
    w = (0.05 * torch.randn(3 * H * 64, D, device=cuda)).bfloat16()
    cos, sin = _rope_tables(geom, 64, cuda)
    col = attn_type == "axial_col"
    q, k, v = C().qkv_rope(h, w, cos, sin, T, S, H, n, col, 0.125)
    qkv = torch.mm(h, w.t()).view(B, n, -1)
    q2, k2, v2 = C().rope_fwd(qkv, cos, sin, T, S, H, col, 0.125)
    for a, b_ in [(q, q2), (k, k2), (v, v2)]:
        assert a.shape == b_.shape
        assert _rel(a, b_) < 1e-2


@pytest.mark.parametrize("M,F,K", [(512, 1024, 256), (2560, 4096, 1024)])
def test_ff_dgrad_geglu_epilogue(cuda, M, F, K):
    """du = dy W2 with the GEGLU backward + FF-in bias grad in the GEMM epilogue == mm + geglu_bwd_bias,
    and both against the fp32 reference."""
    from dalle_amd.ops import hip_ops

    torch.manual_seed(5)
    C = hip_ops.C()
    dy = (torch.randn(M, K, device=cuda) * 0.5).to(torch.bfloat16)
    w2 = torch.randn(K, F, device=cuda) * 0.03  # Linear(F -> K).weight
    h = torch.randn(M, 2 * F, device=cuda).to(torch.bfloat16)
    dh, db = C.ff_dgrad_geglu(dy, w2.t().contiguous().to(torch.bfloat16), h)
    du = torch.mm(dy, w2.to(torch.bfloat16))
    dh_ref, db_ref = C.geglu_bwd_bias(h, du)
    assert _rel(dh, dh_ref) < 1e-2 and _rel(db, db_ref) < 1e-2
    # fp32 reference of the math
    hf = h.float().requires_grad_(True)
    out = hf[:, :F] * torch.nn.functional.gelu(hf[:, F:])
    out.backward(dy.float() @ w2.to(torch.bfloat16).float())
    assert _rel(dh, hf.grad) < 2e-2
    assert _rel(db, hf.grad.sum(0)) < 2e-2
