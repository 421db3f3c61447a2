"""Decode-step skinny GEMM (csrc/kernels/skinny.hip) and its fused epilogues vs fp32 PyTorch references
(MI355X only). Shapes cover one workgroup per column tile (KS = 1) and the cross-workgroup split-K
(last-arriver) path, and batch sizes that are not multiples of 16."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _cnt(device):
    return torch.zeros(8192, dtype=torch.int32, device=device)


SHAPES = [(64, 3072, 1024), (64, 1024, 1024), (48, 1024, 4096), (3, 768, 256), (17, 512, 384), (33, 8192, 1024)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("f32", [False, True])
def test_skinny_linear(cuda, M, N, K, f32):
    from dalle_amd.ops.hip_ops import C

    torch.manual_seed(0)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (0.05 * torch.randn(N, K, device=cuda)).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    cnt = _cnt(cuda)
    want = x.float() @ w.float().t() + b.float()
    for _ in range(3):  # counters must self-reset between launches
        got = C().skinny_linear(x, w, b, f32, cnt)
        assert got.dtype == (torch.float32 if f32 else torch.bfloat16)
        assert _rel(got, want) < 1e-2
    assert int(cnt.abs().sum()) == 0
    got = C().skinny_linear(x, w, None, f32, cnt)
    assert _rel(got, x.float() @ w.float().t()) < 1e-2


def test_skinny_deterministic(cuda):
    from dalle_amd.ops.hip_ops import C

    torch.manual_seed(0)
    x = torch.randn(64, 4096, device=cuda).bfloat16()
    w = torch.randn(1024, 4096, device=cuda).bfloat16()
    cnt = _cnt(cuda)
    a = C().skinny_linear(x, w, None, True, cnt)
    for _ in range(5):
        assert torch.equal(C().skinny_linear(x, w, None, True, cnt), a)


@pytest.mark.parametrize("M,F,K", [(64, 4096, 1024), (5, 1024, 256)])
def test_skinny_geglu(cuda, M, F, K):
    from dalle_amd.ops.hip_ops import C

    torch.manual_seed(0)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (0.05 * torch.randn(2 * F, K, device=cuda)).bfloat16()
    b = torch.randn(2 * F, device=cuda).bfloat16()
    y = x.float() @ w.float().t() + b.float()
    a, g = y.chunk(2, -1)
    want = a * torch.nn.functional.gelu(g)
    got = C().skinny_geglu(x, w, b, _cnt(cuda))
    assert got.shape == (M, F)
    assert _rel(got, want) < 1e-2


@pytest.mark.parametrize("M,N,K", [(64, 1024, 4096), (64, 1024, 1024), (7, 256, 1024)])
def test_skinny_residual(cuda, M, N, K):
    from dalle_amd.ops.hip_ops import C

    torch.manual_seed(0)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (0.05 * torch.randn(N, K, device=cuda)).bfloat16()
    b = torch.randn(N, device=cuda).bfloat16()
    scale = torch.rand(N, device=cuda)
    res = torch.randn(M, N, device=cuda)
    want = res + scale * (x.float() @ w.float().t() + b.float())
    C().skinny_residual_(res, x, w, b, scale, _cnt(cuda))
    assert _rel(res, want) < 1e-3


@pytest.mark.parametrize("M,H", [(64, 16), (3, 4)])
def test_skinny_qkv_rope(cuda, M, H):
    from dalle_amd.ops.hip_ops import C
    from dalle_amd.models.rotary import rotary_tables

    torch.manual_seed(0)
    K, T, S = 64 * H, 17, 8
    n = T + S * S - 1
    cos, sin = rotary_tables(T, S, 64, device=cuda)
    x = torch.randn(M, K, device=cuda).bfloat16()
    w = (0.05 * torch.randn(3 * H * 64, K, device=cuda)).bfloat16()
    pos = torch.tensor(T + 11, dtype=torch.int32, device=cuda)
    q = torch.zeros(M * H, 64, dtype=torch.bfloat16, device=cuda)
    kc = torch.zeros(M * H, n, 64, dtype=torch.bfloat16, device=cuda)
    vc = torch.zeros_like(kc)
    C().skinny_qkv_rope_(x, w, cos, sin, q, kc, vc, pos, H, 0.125, _cnt(cuda))
    # reference: the unfused decode path (GEMM then the decode rotary kernel)
    q2, kc2, vc2 = torch.zeros_like(q), torch.zeros_like(kc), torch.zeros_like(vc)
    qkv = (x.float() @ w.float().t()).bfloat16()
    C().decode_rope_(qkv, cos, sin, q2, kc2, vc2, pos, H, 0.125)
    assert _rel(q, q2) < 1e-2
    assert _rel(kc, kc2) < 1e-2 and _rel(vc, vc2) < 1e-2
    p = int(pos)
    assert kc[:, :p].abs().sum() == 0 and kc[:, p + 1:].abs().sum() == 0
    # past the cache end: no write at all
    pos.fill_(n)
    kc.zero_()
    C().skinny_qkv_rope_(x, w, cos, sin, q, kc, vc, pos, H, 0.125, _cnt(cuda))
    assert kc.abs().sum() == 0


@pytest.mark.parametrize("pattern,pos", [("full", 1100), ("full", 300), ("axial_row", 1000), ("axial_col", 900),
                                         ("conv_like", 700), ("axial_row", 100)])
def test_decode_attention_kernel(cuda, pattern, pos):
    """Decode attention (single-chunk and chunked paths) vs an fp32 softmax over the static mask row."""
    from dalle_amd.models.patterns import AttnGeometry, PATTERN_IDS, static_mask
    from dalle_amd.ops.hip_ops import C

    torch.manual_seed(0)
    T, S, H, B, Ks = 257, 32, 4, 3, 11
    n = T + S * S - 1
    geom = AttnGeometry(T, S, Ks)
    q = torch.randn(B * H, 64, device=cuda).bfloat16()
    kc = torch.randn(B * H, n, 64, device=cuda).bfloat16()
    vc = torch.randn(B * H, n, 64, device=cuda).bfloat16()
    out = torch.zeros(B, H * 64, dtype=torch.bfloat16, device=cuda)
    p = torch.tensor(pos, dtype=torch.int32, device=cuda)
    C().decode_attn_(q, kc, vc, out, p, T, S, H, Ks, PATTERN_IDS[pattern])
    mask = static_mask(geom, pattern, n, device=cuda)[pos, : pos + 1]
    sc = (q.float()[:, None, :] @ kc[:, : pos + 1].float().transpose(1, 2))[:, 0]
    sc = sc.masked_fill(~mask, float("-inf"))
    want = (torch.softmax(sc, -1)[:, None, :] @ vc[:, : pos + 1].float())[:, 0]
    assert _rel(out.view(B * H, 64), want) < 1e-2
