"""CPU golden tests for the model semantics (SURVEY §4 tier 2)."""
import torch
import torch.nn.functional as F
import pytest

from dalle_amd.config import tiny, reference, bench24, DALLEConfig
from dalle_amd.models.dalle import DALLE, layer_scale_init
from dalle_amd.models.patterns import AttnGeometry, static_mask, storage_index
from dalle_amd.models.rotary import rotary_tables, apply_rotary, apply_rotary_inverse, rotary_angles
from dalle_amd.ops import reference as ref

from golden_dalle import axial_attention, conv_attention


def _qkv(bh, n, d, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(bh, n, d, generator=g, dtype=torch.float64) for _ in range(3)]


@pytest.mark.parametrize("T,S", [(65, 16), (9, 8)])
@pytest.mark.parametrize("attn_type", ["axial_row", "axial_col", "conv_like"])
def test_static_mask_matches_golden_sparse_layers(T, S, attn_type):
    geom = AttnGeometry(T, S, 5)
    n = geom.seq_len
    q, k, v = _qkv(3, n + 1, 16)  # golden works on the padded (n+1) sequence
    if attn_type == "conv_like":
        gold = conv_attention(q, k, v, T, S)
    else:
        gold = axial_attention(q, k, v, T, S, 0 if attn_type == "axial_row" else 1)
    gold = gold[:, :n]
    mask = static_mask(geom, attn_type, n)
    scores = torch.einsum("bid,bjd->bij", q[:, :n], k[:, :n]).masked_fill(~mask, -torch.finfo(torch.float64).max)
    out = torch.einsum("bij,bjd->bid", scores.softmax(-1), v[:, :n])
    assert torch.allclose(out, gold, atol=1e-10)


def test_static_mask_structure():
    geom = AttnGeometry(257, 32, 5)
    m = static_mask(geom, "axial_row")
    n = geom.seq_len
    assert m.shape == (n, n)
    assert m[300, :257].all()  # image queries see all text
    assert not m[100, 101]  # text causal
    # image query (row 3, col 5) sees (row 3, cols 0..5) only among image keys
    q = 257 + 3 * 32 + 5
    img_keys = m[q, 257:].nonzero().flatten().tolist()
    assert img_keys == [3 * 32 + c for c in range(6)]
    mc = static_mask(geom, "axial_col")
    img_keys = mc[q, 257:].nonzero().flatten().tolist()
    assert img_keys == [r * 32 + 5 for r in range(4)]
    mv = static_mask(geom, "conv_like")
    img_keys = mv[q, 257:].nonzero().flatten().tolist()
    assert len(img_keys) == 4 * 5  # rows 0..3 (4 rows) x cols 1..5
    st = storage_index(geom, "axial_col")
    assert st[257 + 1].item() == 288 + 32  # image (0,1) stored at column-major slot 1*32+0


def test_token_shift_semantics():
    B, T, S, D = 1, 5, 4, 8
    n = T + S * S - 1
    x = torch.arange(n, dtype=torch.float32).view(1, n, 1).repeat(B, 1, D)
    y = ref.token_shift(x, T, S)
    # text: first half from previous position, pos 0 zeros
    assert (y[0, 0, :4] == 0).all() and (y[0, 3, :4] == 2).all() and (y[0, 3, 4:] == 3).all()
    # image token k=5 (row 1, col 1): top quarter from k=1, left quarter from k=4
    p = T + 5
    assert y[0, p, 0] == T + 1 and y[0, p, 2] == T + 4 and y[0, p, 4] == p
    # image row 0 gets zeros on top quarter, col 0 on left quarter
    assert y[0, T + 2, 0] == 0 and y[0, T + 4, 2] == 0


def test_rotary_tables_and_inverse():
    cos, sin = rotary_tables(257, 32, 64)
    ang = rotary_angles(257, 32, 64)
    assert ang.shape == (257 + 1024, 62)  # 22 text + 40 axial dims rotated
    assert torch.all(cos[:, 62:] == 1) and torch.all(sin[:, 62:] == 0)
    x = torch.randn(2, 1281, 64, dtype=torch.float64)
    c, s = cos.double(), sin.double()
    y = apply_rotary(x, c, s)
    # rotation preserves pair norms
    assert torch.allclose(y.norm(dim=-1), x.norm(dim=-1))
    # inverse is the transpose
    g = torch.randn_like(y)
    lhs = (apply_rotary(x, c, s) * g).sum()
    rhs = (x * apply_rotary_inverse(g, c, s)).sum()
    assert torch.allclose(lhs, rhs)


def test_param_count_matches_reference_recipe():
    cfg = reference()
    m = DALLE(cfg)
    n = sum(p.numel() for p in m.parameters())
    assert n == cfg.unique_param_count() == 125_894_244  # ~125.9M
    assert layer_scale_init(18) == 0.1 and layer_scale_init(19) == 1e-5 and layer_scale_init(25) == 1e-6


def test_state_dict_layout_reversible_and_sequential():
    m = DALLE(tiny(True))
    keys = list(m.state_dict().keys())
    assert "transformer.layers.blocks.0.f.net.fn.fn.fn.to_qkv.weight" in keys
    assert "transformer.layers.blocks.1.g.net.fn.fn.fn.net.3.bias" in keys
    assert "to_logits.1.weight" in keys and "text_emb.linear.weight" in keys
    m2 = DALLE(tiny(False))
    keys2 = list(m2.state_dict().keys())
    assert "transformer.layers.layers.0.0.fn.fn.fn.to_qkv.weight" in keys2
    # tied embeddings: the embedding tables are views of the head
    assert m.text_emb.weight.data_ptr() == m.to_logits[1].weight.data_ptr()


def test_shared_modules_are_aliased():
    cfg = reference()
    m = DALLE(cfg)
    blocks = m.transformer.layers.blocks
    a0 = blocks[0].f.net.fn.fn.fn
    assert a0 is blocks[4].f.net.fn.fn.fn and a0 is not blocks[1].f.net.fn.fn.fn
    assert blocks[63].f.net.fn.fn.fn.attn_type == "conv_like"
    assert blocks[0].f.net.scale is not blocks[4].f.net.scale


def test_loss_matches_masked_full_logits():
    torch.manual_seed(0)
    cfg = tiny(False)
    m = DALLE(cfg)
    text = torch.randint(1, cfg.num_text_tokens, (2, cfg.text_seq_len))
    text[:, 40:] = 0  # unique pad-id remap path
    img = torch.randint(0, cfg.num_image_tokens, (2, cfg.image_seq_len))
    loss = m(text, img, return_loss=True)
    logits = m(text, img, return_loss=False)
    text_bos = m.prepare_text(text)
    labels = torch.cat([text_bos[:, 1:], img + m.num_text_tokens], 1)
    lt = F.cross_entropy(logits[:, : cfg.text_seq_len].reshape(-1, logits.shape[-1]), labels[:, : cfg.text_seq_len].reshape(-1))
    li = F.cross_entropy(logits[:, cfg.text_seq_len:].reshape(-1, logits.shape[-1]), labels[:, cfg.text_seq_len:].reshape(-1))
    assert torch.allclose(loss, (lt + 7 * li) / 8, atol=1e-5)
    assert (text_bos[:, 41:] >= cfg.num_text_tokens).all()  # pads -> unique ids


def test_reversible_grads_match_recomputation():
    """Reversible engine gradients == plain autograd through the same coupling."""
    torch.manual_seed(0)
    cfg = tiny(True)
    m = DALLE(cfg).double()
    text = torch.randint(1, cfg.num_text_tokens, (1, cfg.text_seq_len))
    img = torch.randint(0, cfg.num_image_tokens, (1, cfg.image_seq_len))
    loss = m(text, img, return_loss=True)
    loss.backward()
    g_rev = {n: p.grad.clone() for n, p in m.named_parameters()}
    m.zero_grad()
    # same computation without the custom autograd function
    tr = m.transformer
    from dalle_amd import ops

    def plain(x):
        x1 = x2 = x
        for f, g in tr.layers.pairs():
            x1 = x1 + ops.scale_rows(tr._attn_out(f, x2), f.scale)
            x2 = x2 + ops.scale_rows(tr._ff_out(g, x1), g.scale)
        return (x1 + x2) / 2

    orig = tr.forward
    tr.forward = plain
    try:
        loss2 = m(text, img, return_loss=True)
        loss2.backward()
    finally:
        tr.forward = orig
    assert torch.allclose(loss, loss2)
    for n, p in m.named_parameters():
        assert torch.allclose(p.grad, g_rev[n], atol=1e-8, rtol=1e-6), n


def test_configs():
    c = bench24()
    assert c.depth == 24 and not c.reversible and c.seq_len == 1280
    assert c.train_flops_per_sample() > 3e12
    with pytest.raises(AssertionError):
        DALLEConfig(depth=2, attn_types=["axial_row"], shared_attn_ids=[0, 1], shared_ff_ids=[0, 1])
