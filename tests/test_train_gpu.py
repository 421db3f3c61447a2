"""End-to-end training on MI355X: the tiny DALL-E (BASELINE config 1 geometry) memorises a fixed batch through
the HIP path, and its loss trajectory follows the PyTorch reference ops (same bf16 compute dtype) step by step --
the training-level counterpart of the per-kernel numerics tests. The second test runs the bench engine's own
optimizer path (flat fp32 gradient arena + fused 8-bit LAMB kernel) and checks that it learns."""
import copy

import pytest
import torch

from dalle_amd.config import tiny
from dalle_amd.data.synthetic import synthetic_batch
from dalle_amd.models.dalle import DALLE
from dalle_amd.optim import FlatArena, LAMB8bit

pytestmark = pytest.mark.gpu


def _batch(cfg, dev):
    g = torch.Generator().manual_seed(5)
    return synthetic_batch(4, cfg.text_seq_len, cfg.image_seq_len, cfg.num_text_tokens, cfg.num_image_tokens, g,
                           device=dev)


def _loss(m, b):
    return m(b["input_ids"], b["image"], mask=b["attention_mask"], return_loss=True)


@pytest.mark.parametrize("reversible", [False, True])
def test_hip_training_tracks_reference_ops(cuda, reversible, monkeypatch):
    torch.manual_seed(0)
    cfg = tiny(reversible)
    m0 = DALLE(cfg)
    b = _batch(cfg, cuda)
    runs = {}
    for be in ("auto", "torch"):  # HIP kernels / PyTorch reference ops on the GPU
        monkeypatch.setenv("DALLE_AMD_BACKEND", be)
        m = copy.deepcopy(m0).to(cuda)
        opt = torch.optim.Adam(m.parameters(), lr=3e-3)
        losses = []
        for _ in range(12):
            loss = _loss(m, b)
            opt.zero_grad(set_to_none=True)
            loss.backward()
            opt.step()
            losses.append(loss.item())
        runs[be] = losses
    h, r = runs["auto"], runs["torch"]
    assert all(torch.isfinite(torch.tensor(h)))
    assert h[-1] < 0.5 * h[0], h  # memorising the batch (the reversible stack learns more slowly)
    for i in range(8):  # same trajectory while the losses are O(1)
        assert abs(h[i] - r[i]) <= 0.05 * r[i] + 0.02, (i, h, r)


def test_fused_lamb_arena_training_learns(cuda):
    torch.manual_seed(0)
    cfg = tiny(False)
    m = DALLE(cfg).to(cuda)
    arena = FlatArena(m.parameters(), device=cuda)
    m.grad_arena = arena  # every parameter gradient lands in the fp32 arena inside its producing kernel
    named = list(m.named_parameters())
    groups = [{"params": [p for n, p in named if "bias" not in n], "weight_decay": 0.045},
              {"params": [p for n, p in named if "bias" in n], "weight_decay": 0.0}]
    opt = LAMB8bit(groups, lr=0.01, betas=(0.9, 0.96), eps=1e-6, weight_decay=0.045, clamp_value=10000.0,
                   max_grad_norm=4.0, reuse_grad_buffers=True, optim_bits=8, arena=arena)
    assert opt._get_fused()  # the HIP LAMB kernel over the arena
    b = _batch(cfg, cuda)
    losses = []
    for _ in range(30):
        arena.zero_grad()
        loss = _loss(m, b)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses)))
    assert min(losses[-5:]) < 0.5 * losses[0], losses


def test_grads_reset_between_forward_and_backward(cuda):
    """``loss = model(x); opt.zero_grad(); loss.backward()``: the fused stack was chosen in the forward (every
    parameter had an fp32 .grad), the grads are gone by the backward -- it must still deliver every gradient."""
    torch.manual_seed(0)
    cfg = tiny(False)
    m = DALLE(cfg).to(cuda)
    b = _batch(cfg, cuda)
    _loss(m, b).backward()  # step 1: creates the fp32 .grad buffers
    for p in m.parameters():
        p.grad.zero_()
    _loss(m, b).backward()  # reference: accumulate into zeroed buffers
    ref = {n: p.grad.clone() for n, p in m.named_parameters()}
    loss = _loss(m, b)  # the fused stack sees .grad buffers ...
    for p in m.parameters():
        p.grad = None  # ... that are dropped before the backward
    loss.backward()
    for n, p in m.named_parameters():
        assert p.grad is not None, n
        torch.testing.assert_close(p.grad, ref[n], rtol=1e-4, atol=1e-5, msg=n)


@pytest.mark.parametrize("recompute", [True, False])
def test_reversible_arena_backward_matches_autograd_grads(cuda, recompute):
    """The reversible stack's chained backward (arena sinks: every LayerScale-residual backward fused into the
    LN backward that produces its input grad, rebuilt blocks fetched one step ahead) against the per-op
    backward that returns gradients to autograd (no arena), both from the same weights and batch."""
    torch.manual_seed(0)
    import dataclasses

    cfg = dataclasses.replace(tiny(True), depth=4, attn_types=["axial_row", "axial_col", "axial_row", "conv_like"],
                              shared_attn_ids=[0, 1, 2, 3], shared_ff_ids=[0, 1, 2, 3], reversible_recompute=recompute)
    m = DALLE(cfg).to(cuda)
    b = _batch(cfg, cuda)
    _loss(m, b).backward()  # plain autograd grads (no .grad buffers existed in the forward)
    ref = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad(set_to_none=True)
    arena = FlatArena(m.parameters(), device=cuda)
    m.grad_arena = arena
    arena.zero_grad()
    _loss(m, b).backward()
    for n, p in m.named_parameters():
        torch.testing.assert_close(p.grad, ref[n], rtol=2e-3, atol=2e-5, msg=n)
