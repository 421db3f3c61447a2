"""Randomised property tests (hypothesis, SURVEY §4 tier 1/3): blockwise quantisation, the
averaging compressions, butterfly shard partitions, the sparse attention masks against their
brute-force definitions (ragged text lengths), and the flat arena layout."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from dalle_amd.models.patterns import AttnGeometry, static_mask
from dalle_amd.optim import FlatArena, quant
from dalle_amd.parallel.averaging import shard_bounds
from dalle_amd.parallel.compression import Float16Compression, Uniform8BitQuantization

FAST = settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])


@FAST
@given(n=st.integers(1, 3 * 4096 + 77), scale=st.floats(1e-6, 1e3), signed=st.booleans(), seed=st.integers(0, 2 ** 16))
def test_blockwise_quant_nearest_code_and_block_absmax(n, scale, signed, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g) * scale
    if not signed:
        x = x.abs()
    code = quant.dynamic_map(signed)
    q, absmax = quant.quantize_blockwise(x, code)
    assert q.dtype == torch.uint8 and absmax.numel() == quant.num_blocks(n)
    ref_absmax = torch.stack([b.abs().max() for b in x.split(quant.BLOCK)])
    assert torch.equal(absmax, ref_absmax)
    normed = x / absmax.repeat_interleave(quant.BLOCK)[:n].clamp_min(1e-30)
    err_best = (code[None, :] - normed[:, None]).abs().min(dim=1).values
    assert torch.allclose((code[q.long()] - normed).abs(), err_best, atol=1e-6)
    y = quant.dequantize_blockwise(q, absmax, code)
    # the dynamic map's largest relative gap is < 10% of the block max
    assert ((y - x).abs() <= 0.1 * absmax.repeat_interleave(quant.BLOCK)[:n] + 1e-30).all()


@FAST
@given(n=st.integers(2, 50_000), seed=st.integers(0, 2 ** 16), shift=st.floats(-5, 5))
def test_uniform8bit_codebook_is_bin_mean(n, seed, shift):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, generator=g) + shift
    u = Uniform8BitQuantization()
    c = u.compress(x)
    idx, book = c["idx"].long(), c["codebook"]
    assert book.shape == (256,)
    for b in idx.unique()[:16].tolist():
        assert torch.allclose(book[b], x[idx == b].mean(), rtol=1e-4, atol=1e-5)
    # dequantisation never moves a value farther than its own bin's spread
    y = u.roundtrip(x)
    assert y.shape == x.shape and torch.isfinite(y).all()


@FAST
@given(x=st.lists(st.floats(-7e4, 7e4, allow_nan=False, width=32), min_size=1, max_size=300))
def test_fp16_compression_clamps_and_rounds(x):
    t = torch.tensor(x, dtype=torch.float32)
    y = Float16Compression().roundtrip(t)
    assert torch.equal(y, t.clamp(-65504, 65504).half().float())


@FAST
@given(numel=st.integers(0, 10 ** 7), w=st.lists(st.sampled_from([0.0, 1.0, 0.5, 2.0]), min_size=1, max_size=8))
def test_shard_bounds_partition(numel, w):
    if sum(w) == 0:
        w = w[:-1] + [1.0]
    b = shard_bounds(numel, w)
    assert len(b) == len(w) + 1 and b[0] == 0 and b[-1] == numel
    assert all(lo <= hi for lo, hi in zip(b[:-1], b[1:]))
    for wi, lo, hi in zip(w, b[:-1], b[1:]):
        if wi == 0:
            assert lo == hi  # client-mode peers host no shard


def _brute_force_allowed(T, S, attn_type, i, j):
    """The reference semantics written out per (query i, key j) on the 1-D sequence."""
    if j > i:
        return False
    if i < T or j < T:  # text queries: causal; every image query sees all text keys
        return j < T or i < T and j <= i
    ri, ci = divmod(i - T, S)
    rj, cj = divmod(j - T, S)
    if attn_type == "full":
        return True
    if attn_type == "axial_row":
        return ri == rj and cj <= ci
    if attn_type == "axial_col":
        return ci == cj and rj <= ri
    # conv_like: upper-left 5x5 window incl. self (causal padding)
    return 0 <= ri - rj <= 4 and 0 <= ci - cj <= 4 and (rj, cj) <= (ri, ci)


@settings(max_examples=12, deadline=None)
@given(T=st.integers(1, 70), S=st.sampled_from([4, 8, 16]),
       attn_type=st.sampled_from(["full", "axial_row", "axial_col", "conv_like"]))
def test_static_masks_match_definition(T, S, attn_type):
    geom = AttnGeometry(T, S, 5)
    n = geom.seq_len
    m = static_mask(geom, attn_type, n)
    want = torch.tensor([[_brute_force_allowed(T, S, attn_type, i, j) for j in range(n)] for i in range(n)])
    assert torch.equal(m.cpu(), want)


@FAST
@given(shapes=st.lists(st.tuples(st.integers(1, 70), st.integers(1, 130)), min_size=1, max_size=6))
def test_flat_arena_alignment_and_views(shapes):
    ps = [torch.nn.Parameter(torch.randn(*s)) for s in shapes]
    vals = [p.detach().clone() for p in ps]
    a = FlatArena(ps)
    for p, v, o in zip(ps, vals, a.offsets):
        assert o % a.align == 0
        assert torch.equal(p.detach(), v)
        assert p.data.data_ptr() == a.data[o:].data_ptr() and p.grad.data_ptr() == a.grad[o:].data_ptr()
    blocks = a.block_tensor.tolist()
    for i, (p, o) in enumerate(zip(ps, a.offsets)):
        nb = -(-p.numel() // a.align)
        assert blocks[o // a.align: o // a.align + nb] == [i] * nb
    assert np.isclose(a.data.sum().item(), sum(v.sum().item() for v in vals), rtol=1e-4, atol=1e-3)
