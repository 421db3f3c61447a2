"""The hand-scheduled assembly GEMM (csrc/asm/gen_gemm.py, ``_C.asm_gemm``) against an fp32 PyTorch product:
plain and fp32-bias epilogues, several tile / K-step counts (the K-step schedule's first / loop / penultimate /
last iterations, persistent workgroups walking several tiles -- with a column-index carry when the grid is
not a multiple of the tile columns -- with immediate (4 K-steps) and deferred epilogue stores), strided operand rows and an output view."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    from dalle_amd.ops.ext import load_extension

    return load_extension(required=True)


@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (512, 768, 384), (2560, 1024, 1024), (4096, 3072, 1024),
                                   (2560, 1024, 4096), (8192, 256, 512), (65536, 1024, 256),
                                   (25600, 768, 384), (25600, 768, 1024)])
@pytest.mark.parametrize("bias", [False, True])
def test_asm_gemm_matches_fp32(cuda, C, M, N, K, bias):
    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    B = torch.randn(N, K, device=cuda).to(torch.bfloat16)
    b = torch.randn(N, device=cuda) if bias else None
    ref = A.float() @ B.float().t() + (b if bias else 0)
    got = C.asm_gemm(A, B, b, None).float()
    err = ((got - ref).abs().max() / ref.abs().max()).item()
    assert err < 8e-3, err
    assert torch.equal(C.asm_gemm(A, B, b, None), C.asm_gemm(A, B, b, None))  # deterministic


def test_asm_gemm_strided_rows_and_out_view(cuda, C):
    torch.manual_seed(1)
    M, N, K = 1024, 512, 512
    Abig = torch.randn(M, K + 128, device=cuda).to(torch.bfloat16)
    Bbig = torch.randn(N, K + 64, device=cuda).to(torch.bfloat16)
    A, B = Abig[:, 64:64 + K], Bbig[:, :K]
    out = torch.full((M, N + 256), 7.0, device=cuda, dtype=torch.bfloat16)
    C.asm_gemm(A, B, None, out[:, 256:])
    ref = A.float() @ B.float().t()
    err = ((out[:, 256:].float() - ref).abs().max() / ref.abs().max()).item()
    assert err < 8e-3, err
    assert torch.all(out[:, :256] == 7.0)   # nothing outside the view is written


def test_asm_gemm_rejects_untiled(cuda, C):
    A = torch.randn(300, 256, device=cuda).to(torch.bfloat16)
    B = torch.randn(256, 256, device=cuda).to(torch.bfloat16)
    with pytest.raises(RuntimeError):
        C.asm_gemm(A, B, None, None)


@pytest.mark.parametrize("Ktot,M,N,splits", [(2048, 256, 256, 1), (4096, 512, 768, 2), (16384, 1024, 1024, 16),
                                             (24576, 768, 512, 3), (32768, 3072, 1024, 16)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_asm_wgrad_matches_fp32(cuda, C, Ktot, M, N, splits, accumulate):
    """dW (+)= G^T X on the assembly TN kernel (token-major operands, split-K partial slabs + fold)"""
    torch.manual_seed(Ktot + M + N)
    G = torch.randn(Ktot, M, device=cuda).to(torch.bfloat16)
    X = torch.randn(Ktot, N, device=cuda).to(torch.bfloat16)
    out = torch.randn(M, N, device=cuda)
    init = out.clone()
    C.asm_wgrad_(out, G, X, splits, accumulate)
    ref = G.float().t() @ X.float() + (init if accumulate else 0)
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-4, err


def test_weight_grad_routes_to_asm(cuda, C):
    from dalle_amd.ops import hip_ops

    if not hip_ops.ASM_GEMM:
        pytest.skip("assembly GEMM disabled")
    torch.manual_seed(3)
    w = torch.nn.Parameter(torch.randn(1024, 1024, device=cuda))
    w.grad = torch.zeros_like(w)
    g = torch.randn(8192, 1024, device=cuda).to(torch.bfloat16)
    x = torch.randn(8192, 1024, device=cuda).to(torch.bfloat16)
    before = hip_ops.PATH_COUNTS.get("asm_wgrad", 0)
    assert hip_ops.weight_grad(w, g, x) is None
    ref = g.float().t() @ x.float()
    assert ((w.grad - ref).abs().max() / ref.abs().max()).item() < 1e-4
    assert hip_ops.PATH_COUNTS.get("asm_wgrad", 0) == before + 1


@pytest.mark.parametrize("M,F,K", [(512, 1024, 1024), (10240, 4096, 1024), (2560, 512, 1024), (5120, 8192, 2048)])
def test_asm_ff_in_geglu(cuda, C, M, F, K):
    """FF-in GEMM + GEGLU in one assembly kernel (permuted W1 rows, u from the stored bf16 pre-activation,
    deferred under the next tile's K-steps): a vs fp32 x W1^T + b1, u vs the unfused GEGLU of that a."""
    from dalle_amd.ops import hip_ops

    torch.manual_seed(M + F)
    x = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w1 = torch.randn(2 * F, K, device=cuda) * 0.03
    b1 = torch.randn(2 * F, device=cuda) * 0.1
    a, u = hip_ops.ff_in_geglu(x, w1, b1)
    ref_a = x.float() @ w1.to(torch.bfloat16).float().t() + b1
    assert ((a.float() - ref_a).abs().max() / ref_a.abs().max()).item() < 8e-3
    af = a.float()
    ref_u = af[:, :F] * torch.nn.functional.gelu(af[:, F:])
    assert ((u.float() - ref_u).abs().max() / ref_u.abs().max()).item() < 8e-3
    assert torch.equal(u, C.geglu_fwd(a)) or ((u.float() - C.geglu_fwd(a).float()).abs().max() <= 2 ** -6 * ref_u.abs().max())


@pytest.mark.parametrize("B,H", [(2, 16), (8, 16), (8, 32)])
@pytest.mark.parametrize("col", [False, True])
def test_asm_qkv_rope_matches_separate_path(cuda, C, col, B, H):
    """QKV projection + 3-axis rotary on the assembly kernel (rotation deferred onto the stored bf16 values) ==
    the unfused path (the projection, then rope_fwd on its bf16 output) on the reference geometry
    (257 text + 32x32 image tokens, 16 heads: tiles straddle the text / image boundary). Two samples = 120
    tiles, one per workgroup (the straight final path); eight = 480 tiles, so workgroups walk several tiles
    and rotate / store under the successor tile's K-steps."""
    from dalle_amd.models.patterns import AttnGeometry
    from dalle_amd.ops.hip_ops import _cs3_from_tables, _rope_tables

    torch.manual_seed(7)
    T, S = 257, 32
    d = H * 64          # 16 heads: d_model 1024 (K-steps 0..13 unrolled + tail); 32 heads: d_model 2048 (+ 16 looped)
    n = T + S * S - 1
    geom = AttnGeometry(T, S, 5)
    h = torch.randn(B * n, d, device=cuda).to(torch.bfloat16)
    w = (torch.randn(3 * H * 64, d, device=cuda) * 0.03).to(torch.bfloat16)
    cos, sin = _rope_tables(geom, 64, cuda)
    q, k, v = C.asm_qkv_rope(h, w, _cs3_from_tables(cos, sin, 0.125), T, S, H, n, col)
    qkv = (h.float() @ w.float().t()).to(torch.bfloat16).view(B, n, -1)
    q2, k2, v2 = C.rope_fwd(qkv, cos, sin, T, S, H, col, 0.125)
    for a, b in ((q, q2), (k, k2), (v, v2)):
        assert a.shape == b.shape
        err = ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()
        assert err < 1e-2, err


@pytest.mark.parametrize("M,F,K", [(512, 256, 1024), (2560, 1024, 1024), (20480, 4096, 1024), (10240, 8192, 2048)])
def test_asm_ff_dgrad_geglu(cuda, C, M, F, K):
    """FF-out dgrad + GEGLU backward + FF-in bias column sums on the assembly kernel vs fp32: du = bf16(dy W2),
    da_value = du gelu(gate), da_gate = du value gelu'(gate) (exact erf GELU), db = column sums of (da_value,
    da_gate). 20480 x 4096 = 1280 tiles: workgroups walk several (the deferred path)."""
    torch.manual_seed(M + F)
    dy = torch.randn(M, K, device=cuda).to(torch.bfloat16)
    w2t = (torch.randn(F, K, device=cuda) * 0.03).to(torch.bfloat16)
    h = torch.randn(M, 2 * F, device=cuda).to(torch.bfloat16)
    dh, db = C.asm_ff_dgrad_geglu(dy, w2t, h, None)
    du = (dy.float() @ w2t.float().t()).to(torch.bfloat16).float()
    v, g = h.float()[:, :F], h.float()[:, F:]
    cdf = 0.5 * (1 + torch.erf(g * 0.7071067811865476))
    pdf = torch.exp(-0.5 * g * g) * 0.3989422804014327
    ref = torch.cat([du * g * cdf, du * v * (cdf + g * pdf)], 1)
    assert ((dh.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    ref_db = ref.sum(0)
    assert ((db - ref_db).abs().max() / ref_db.abs().max()).item() < 1e-2
    dh2, db2 = C.ff_dgrad_geglu(dy, w2t, h, None)       # the HIP kernel it replaces
    assert ((dh.float() - dh2.float()).abs().max() / ref.abs().max()).item() < 1e-2
