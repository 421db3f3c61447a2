"""Persistent GEMM family (csrc/kernels/gemm_pt.hip) against fp32 PyTorch references: the plain bf16
product (+bias), QKV + 3-axis rotary into the attention storage, the FF-in GEMM + GEGLU forward and the
FF-out dgrad + GEGLU backward. Shapes cover one tile per workgroup, several tiles per workgroup (the
continuous cross-tile DMA stream), the XCD remap (tile count % 8 == 0) and its absence."""
import pytest
import torch

from dalle_amd.models.patterns import AttnGeometry

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def test_permlane16_swap_convention(cuda):
    """The epilogues assume v_permlane16_swap trades rows 1, 3 of its first operand with rows 0, 2 of
    its second (rows = 16 lanes)."""
    from dalle_amd.ops.hip_ops import C

    out = C().permlane16_probe().cpu().tolist()
    x, y = out[:64], out[64:]
    lane = list(range(64))
    want_x = [l if (l >> 4) % 2 == 0 else 100 + l - 16 for l in lane]
    want_y = [l + 16 if (l >> 4) % 2 == 0 else 100 + l for l in lane]
    assert x == want_x and y == want_y


SHAPES = [(256, 256, 128), (512, 768, 320), (2048, 1024, 192), (4096, 2048, 256), (8192, 8192, 128), (8192, 4096, 192),
          (61440 // 8, 3072, 1024)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("group", [0, 2, -3])
@pytest.mark.parametrize("variant", [10, 20])  # one tile per workgroup | persistent
def test_gemm_pt(cuda, M, N, K, group, variant):
    from dalle_amd.ops.hip_ops import C

    torch.manual_seed(0)
    A = torch.randn(M, K, device=cuda).bfloat16()
    B = torch.randn(N, K, device=cuda).bfloat16()
    bias = torch.randn(N, device=cuda).bfloat16()
    ref = A.float() @ B.float().t()
    got = C().gemm_pt(A, B, bias, variant, group)
    assert _rel(got, ref + bias.float()) < 5e-3
    got = C().gemm_pt(A, B, None, variant, group)
    assert _rel(got, ref) < 5e-3
    # every element is written (catch a missed tile / sub-tile): compare elementwise with a loose bound
    assert ((got.float() - ref).abs() <= 0.02 * ref.abs() + 0.5).all()
    # deterministic
    assert torch.equal(got, C().gemm_pt(A, B, None, variant, group))


@pytest.mark.parametrize("attn_type", ["axial_row", "axial_col", "conv_like"])
@pytest.mark.parametrize("persist", [0, 1])
def test_qkv_rope_pt(cuda, attn_type, persist):
    from dalle_amd.ops.hip_ops import C, _rope_tables, rope_cs_table

    torch.manual_seed(0)
    T, S, H, D = 65, 16, 4, 256
    geom = AttnGeometry(T, S, 5)
    n, B = T + S * S - 1, 8  # M = 2560: several tiles per workgroup on small grids
    h = torch.randn(B * n, D, device=cuda).bfloat16()
    w = (0.05 * torch.randn(3 * H * 64, D, device=cuda)).bfloat16()
    cos, sin = _rope_tables(geom, 64, cuda)
    col = attn_type == "axial_col"
    q, k, v = C().qkv_rope_pt(h, w, rope_cs_table(geom, 64, cuda), T, S, H, n, col, 0.125, persist)
    qkv = (h.float() @ w.float().t()).view(B, n, -1)
    # storage-layout reference: the unfused rotary kernel on the bf16-rounded product (the fused kernel
    # rotates in fp32 and rounds once, so the two differ by at most about one bf16 ulp)
    q2, k2, v2 = C().rope_fwd(qkv.bfloat16(), cos, sin, T, S, H, col, 0.125)
    for got, ref in [(q, q2), (k, k2), (v, v2)]:
        assert got.shape == ref.shape
        assert _rel(got, ref) < 1e-2
        # every element mapped (a wrong row / head / pair would be off by O(max)); rounding differences of
        # the cancelling rotary sums are bounded by the operands' scale, not the result's
        assert ((got.float() - ref.float()).abs() <= 0.02 * ref.float().abs().max()).all()


@pytest.mark.parametrize("M,F,K", [(512, 1024, 256), (2560, 4096, 1024)])
@pytest.mark.parametrize("persist", [0, 1])
def test_ff_dgrad_geglu_pt(cuda, M, F, K, persist):
    from dalle_amd.ops import hip_ops

    torch.manual_seed(5)
    C = hip_ops.C()
    dy = (torch.randn(M, K, device=cuda) * 0.5).to(torch.bfloat16)
    w2 = torch.randn(K, F, device=cuda) * 0.03
    h = torch.randn(M, 2 * F, device=cuda).to(torch.bfloat16)
    w2t = w2.t().contiguous().to(torch.bfloat16)
    dh, db = C.ff_dgrad_geglu_pt(dy, w2t, h, None, persist)
    dh_old, db_old = C.ff_dgrad_geglu(dy, w2t, h)
    assert _rel(dh, dh_old) < 1e-2 and _rel(db, db_old) < 1e-2
    if persist == 0:
        # one tile per workgroup: the 8-phase kernel's LDS-staged epilogue on the same bf16 du -- equal up to
        # the compiler's contraction of the GELU multiply-adds (one bf16 ulp); bias sums in another order
        assert ((dh.float() - dh_old.float()).abs() <= 2 ** -7 * dh_old.float().abs() + 1e-6).all()
        assert _rel(db, db_old) < 1e-5
    hf = h.float().requires_grad_(True)
    out = hf[:, :F] * torch.nn.functional.gelu(hf[:, F:])
    out.backward(dy.float() @ w2.to(torch.bfloat16).float())
    assert _rel(dh, hf.grad) < 2e-2
    assert _rel(db, hf.grad.sum(0)) < 2e-2
    # bias-grad accumulation into a sink
    sink = torch.ones(2 * F, device=cuda)
    C.ff_dgrad_geglu_pt(dy, w2t, h, sink, persist)
    assert _rel(sink - 1, db) < 1e-5


@pytest.mark.parametrize("cpol", [0, 1, 2, 16, 17])
@pytest.mark.parametrize("drain", [0, 1])
def test_store_policy_and_drain_bitwise(cuda, cpol, drain):
    """Output-store cache policies (gemm_set_cpol: plain / sc0 / nt / sc1 / sc0 sc1 buffer stores) and the
    end-of-workgroup store drain (gemm_set_drain) change how the epilogue writes, never what: every
    hand-written GEMM form is bitwise equal to the plain-store, no-drain result."""
    from dalle_amd.ops import hip_ops

    C = hip_ops.C()
    torch.manual_seed(1)
    M, N, K = 2048, 1024, 256
    A = torch.randn(M, K, device=cuda).bfloat16()
    B = torch.randn(N, K, device=cuda).bfloat16()
    bias = torch.randn(N, device=cuda).bfloat16()
    dy = (0.5 * torch.randn(M, K, device=cuda)).bfloat16()
    w2t = (0.05 * torch.randn(N, K, device=cuda)).bfloat16()
    a = torch.randn(M, 2 * N, device=cuda).bfloat16()

    def run_all():
        outs = [C.gemm_pt(A, B, bias, 10, 0), C.gemm_pt(A, B, bias, 20, 0), C.gemm_nt(A, B, None, 300)]
        dh8 = C.ff_dgrad_geglu(dy, w2t, a, None, 0)
        dhp = C.ff_dgrad_geglu_pt(dy, w2t, a)
        outs += list(dh8) if isinstance(dh8, (tuple, list)) else [dh8]
        outs += list(dhp) if isinstance(dhp, (tuple, list)) else [dhp]
        return [o.clone() for o in outs]

    try:
        C.gemm_set_cpol(0)
        C.gemm_set_drain(0)
        ref = run_all()
        C.gemm_set_cpol(cpol)
        C.gemm_set_drain(drain)
        got = run_all()
    finally:
        C.gemm_set_cpol(0)
        C.gemm_set_drain(1)
    for r, g in zip(ref, got):
        assert torch.equal(r, g)


@pytest.mark.parametrize("M,F,K", [(512, 1024, 256), (2560, 4096, 1024)])
def test_ff_dgrad_geglu_two_workgroup_bitwise(cuda, M, F, K):
    """The two-workgroups-per-CU FF-out dgrad + GEGLU backward (gemm_set_geglu_bwd_2wg) walks K in the same
    32-deep chunks as the 8-phase kernel and shares its epilogue: bitwise equal dh and bias partials. The
    plain two-workgroup product against an fp32 reference."""
    from dalle_amd.ops import hip_ops

    C = hip_ops.C()
    torch.manual_seed(13)
    dy = (torch.randn(M, K, device=cuda) * 0.5).bfloat16()
    w2t = (torch.randn(F, K, device=cuda) * 0.03).bfloat16()
    h = torch.randn(M, 2 * F, device=cuda).bfloat16()
    try:
        C.gemm_set_geglu_bwd_2wg(0)
        dh0, db0 = C.ff_dgrad_geglu(dy, w2t, h)
        C.gemm_set_geglu_bwd_2wg(1)
        dh1, db1 = C.ff_dgrad_geglu(dy, w2t, h)
    finally:
        C.gemm_set_geglu_bwd_2wg(0)
    assert torch.equal(dh0, dh1) and torch.equal(db0, db1)
    got = C.gemm_2wg(dy, w2t)
    assert _rel(got, dy.float() @ w2t.float().t()) < 5e-3
