"""hipBLASLt strided-batched bf16 -> fp32 product with a measured solution (csrc/blaslt/lt_tuned.cpp) on the
split-K weight-gradient views of hip_ops._weight_grad_t: equal to torch.bmm up to fp32 summation order,
deterministic after the search."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _views(form, M, N, K, s, dev):
    g2 = torch.randn(M, N, device=dev).bfloat16()
    x2 = torch.randn(M, K, device=dev).bfloat16()
    ms = M // s
    gt, xt = g2.t().contiguous(), x2.t().contiguous()
    a = gt.view(N, s, ms).transpose(0, 1) if form in ("gt", "nt") else g2.view(s, ms, N).transpose(1, 2)
    b = xt.view(K, s, ms).transpose(0, 1).transpose(1, 2) if form in ("xt", "nt") else x2.view(s, ms, K)
    return a, b


@pytest.mark.parametrize("form", ["xt", "gt", "nt", "plain"])
@pytest.mark.parametrize("N,K,s", [(256, 512, 4), (384, 128, 2)])
def test_lt_bmm_matches_torch_bmm(cuda, form, N, K, s):
    from dalle_amd.ops import hip_ops

    C = hip_ops.C()
    torch.manual_seed(21)
    a, b = _views(form, 4096, N, K, s, cuda)
    ref = torch.bmm(a, b, out_dtype=torch.float32)
    out = torch.empty(s, N, K, device=cuda)
    idx = C.lt_bmm_(a, b, out, True, 1)
    assert idx >= 0
    assert ((out - ref).norm() / ref.norm()).item() < 1e-5
    again = torch.empty_like(out)
    assert C.lt_bmm_(a, b, again, True, 1) == idx
    assert torch.equal(out, again)
