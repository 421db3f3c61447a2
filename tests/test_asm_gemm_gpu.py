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
