"""Fused decode sampler (csrc/kernels/sample.hip) vs the PyTorch filter semantics of
``dalle_amd.models.generation.filter_logits``: kept sets, greedy limit, sampling distribution and the
decode-step bookkeeping (MI355X only)."""
import pytest
import torch

from dalle_amd.models.generation import filter_logits

pytestmark = pytest.mark.gpu


def _C():
    from dalle_amd.ops.hip_ops import C

    return C()


def _run(logits, top_k, top_p, temperature, seed, pos=0):
    dev = logits.device
    s = torch.tensor(seed, dtype=torch.int64, device=dev)
    p = torch.tensor(pos, dtype=torch.int32, device=dev)
    return _C().sample_step(logits.contiguous(), top_k, top_p, temperature, s, p)


@pytest.mark.parametrize("top_k,top_p", [(0, 1.0), (256, 1.0), (1, 1.0), (0, 0.9), (256, 0.8), (50, 0.3), (8192, 0.95)])
def test_samples_stay_in_the_filtered_set(cuda, top_k, top_p):
    torch.manual_seed(0)
    B, V = 16, 8192
    logits = torch.randn(B, V, device=cuda) * 3
    kept = torch.isfinite(filter_logits(logits, top_k, top_p))
    for seed in range(20):
        nxt = _run(logits, top_k, top_p, 1.0, seed)
        assert nxt.dtype == torch.int64 and nxt.shape == (B,)
        assert kept.gather(1, nxt.view(B, 1)).all(), (top_k, top_p, seed)
    # greedy limit = argmax of the filtered logits
    g = _run(logits, top_k, top_p, 0.0, 123)
    assert torch.equal(g, logits.argmax(-1))


@pytest.mark.parametrize("top_k,top_p", [(0, 1.0), (5, 1.0), (0, 0.7)])
def test_sampling_distribution(cuda, top_k, top_p):
    V, n = 16, 8192  # n rows of the same logits = n independent draws (the hash includes the row)
    base = torch.linspace(-2.0, 1.5, V, device=cuda)
    logits = base.repeat(n, 1)
    temperature = 0.8
    want = torch.softmax(filter_logits(base.view(1, V), top_k, top_p) / temperature, -1).view(V)
    got = torch.zeros(V, device=cuda)
    for seed in range(4):
        got += torch.bincount(_run(logits, top_k, top_p, temperature, 1000 + seed), minlength=V).float()
    got /= got.sum()
    assert (got[want == 0] == 0).all()
    assert (got - want).abs().max().item() < 0.015, (got, want)


def test_ragged_vocab_and_ties(cuda):
    V = 1000  # not a multiple of the block
    logits = torch.zeros(3, V, device=cuda)
    logits[:, 10] = logits[:, 500] = logits[:, 999] = 5.0  # a 3-way tie at the top
    for seed in range(10):
        nxt = _run(logits, 2, 1.0, 1.0, seed)  # ties at the k-th value are kept (torch semantics)
        assert set(nxt.tolist()) <= {10, 500, 999}
    assert _run(logits, 0, 1.0, 0.0, 0).tolist() == [10, 10, 10]  # greedy ties -> smallest index


def test_decode_bookkeeping(cuda):
    B, T, img, vt = 4, 6, 9, 1000
    text = torch.randint(2, 900, (B, T), device=cuda)
    codes = torch.full((B, img), -1, dtype=torch.int64, device=cuda)
    tok = torch.zeros(B, dtype=torch.int64, device=cuda)
    seed = torch.tensor(5, dtype=torch.int64, device=cuda)
    logits = torch.randn(B, 64, device=cuda)
    C = _C()
    for pos in range(T + img - 1):
        p = torch.tensor(pos, dtype=torch.int32, device=cuda)
        nxt = C.sample_step(logits, 0, 1.0, 1.0, seed, p, text, codes, tok, vt)
        if pos + 1 < T:
            assert torch.equal(tok, text[:, pos + 1])
        else:
            assert torch.equal(tok, nxt + vt)
            assert torch.equal(codes[:, pos - T + 1], nxt)
    assert (codes >= 0).all() and (codes < 64).all()
    # same seed + position -> same draw (replay-safe); another position -> fresh noise
    p = torch.tensor(7, dtype=torch.int32, device=cuda)
    a = C.sample_step(logits, 0, 1.0, 1.0, seed, p)
    b = C.sample_step(logits, 0, 1.0, 1.0, seed, p)
    assert torch.equal(a, b)
