"""HIP decode path (decode LN-shift / rotary-into-cache / sparse decode attention, hipGraph) on MI355X."""
import pytest
import torch

from dalle_amd.config import DALLEConfig, tiny
from dalle_amd.models.dalle import DALLE
from dalle_amd.models.generation import DecodeEngine
from dalle_amd.models.vqgan import VQGanVAE

pytestmark = pytest.mark.gpu


def _cfg(reversible):
    c = tiny(reversible)
    return DALLEConfig(**{**c.to_dict(), "depth": 4, "attn_types": ["axial_row", "axial_col", "conv_like", "full"],
                          "shared_attn_ids": [0, 1, 2, 3], "shared_ff_ids": [0, 1, 0, 1]})


@pytest.mark.parametrize("skinny", ["1", "0", "handoff", "residual_partials"])
@pytest.mark.parametrize("reversible", [False, True])
def test_hip_decode_matches_reference_decode(cuda, reversible, skinny):
    """``1``: every projection as split-K slabs summed by its consumer (default); ``handoff``: in-GEMM
    split-K hand-off; ``residual_partials``: slabs for the residual projections only."""
    partials = {"handoff": 0, "residual_partials": 1}.get(skinny, 2)
    skinny = "1" if skinny in ("handoff", "residual_partials") else skinny
    torch.manual_seed(0)
    cfg = _cfg(reversible)
    m = DALLE(cfg).eval()
    B = 3
    text = torch.randint(2, cfg.num_text_tokens, (B, cfg.text_seq_len))
    img = torch.randint(0, cfg.num_image_tokens, (B, cfg.image_seq_len))
    ref = DecodeEngine(m, B, device=torch.device("cpu"), use_hip=False).teacher_forced_logits(m.prepare_text(text), img)
    mg = m.to(cuda)
    eng = DecodeEngine(mg, B, device=cuda, use_hip=True, skinny=skinny == "1", partials=partials)
    assert eng.skinny == (skinny == "1")
    out = eng.teacher_forced_logits(mg.prepare_text(text.to(cuda)), img.to(cuda)).cpu()
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 3e-2, rel
    # argmax agreement on the vast majority of positions
    agree = (out.argmax(-1) == ref.argmax(-1)).float().mean().item()
    assert agree > 0.9, agree


def test_graph_replay_matches_eager(cuda):
    torch.manual_seed(0)
    cfg = _cfg(False)
    m = DALLE(cfg).eval().to(cuda)
    text = torch.randint(2, cfg.num_text_tokens, (2, cfg.text_seq_len), device=cuda)
    eager = m.generate_images(text, temperature=1e-6, use_graph=False)
    graph = m.generate_images(text, temperature=1e-6, use_graph=True)
    assert torch.equal(eager, graph)


@pytest.mark.parametrize("use_graph,graphs", [(False, "per-part"), (True, "per-part"), (True, "joint")])
def test_split_decode_engine_matches_single(cuda, use_graph, graphs):
    """Two half-batch chains on separate streams (per-part graphs, or one graph with the chains as branches)
    == one full-batch engine under greedy sampling (top-k 1: the sampler's noise, which differs per part,
    cannot change the pick)."""
    from dalle_amd.models.generation import SplitDecodeEngine

    torch.manual_seed(0)
    cfg = _cfg(False)
    m = DALLE(cfg).eval().to(cuda)
    B = 4
    text = torch.randint(2, cfg.num_text_tokens, (B, cfg.text_seq_len), device=cuda)
    tb = m.prepare_text(text)
    single = DecodeEngine(m, B, device=cuda).generate(tb, top_k=1, use_graph=use_graph, seed=5)
    split = SplitDecodeEngine(m, B, device=cuda, parts=2, graphs=graphs)
    assert len(split.parts) == 2 and split.parts[1]._w is split.parts[0]._w
    got = split.generate(tb, top_k=1, use_graph=use_graph, seed=5)
    assert got.shape == single.shape
    assert (got == single).float().mean().item() > 0.98
    # a second call reuses the captured graph and the shared weights
    again = split.generate(tb, top_k=1, use_graph=use_graph, seed=7)
    assert torch.equal(again, got)


def test_split_decode_per_part_graphs_equal_joint_graph(cuda):
    """The per-part graphs (each part's step a linear graph on its own stream) run the same kernels on the same
    buffers as the joint two-branch graph: bitwise the same codes under top-k sampling with a fixed seed, and
    the same as the eager steps."""
    from dalle_amd.models.generation import SplitDecodeEngine

    torch.manual_seed(0)
    cfg = _cfg(True)
    m = DALLE(cfg).eval().to(cuda)
    B = 8
    text = torch.randint(2, cfg.num_text_tokens, (B, cfg.text_seq_len), device=cuda)
    tb = m.prepare_text(text)
    out = {}
    for graphs in ("per-part", "joint"):
        eng = SplitDecodeEngine(m, B, device=cuda, parts=2, graphs=graphs)
        assert eng.graph_mode == graphs
        out[graphs] = eng.generate(tb, top_k=16, use_graph=True, seed=11)
        out[graphs + "-eager"] = eng.generate(tb, top_k=16, use_graph=False, seed=11)
    assert torch.equal(out["per-part"], out["joint"])
    assert torch.equal(out["per-part"], out["per-part-eager"])
    with pytest.raises(ValueError):
        SplitDecodeEngine(m, B, device=cuda, parts=2, graphs="bogus")


def test_parallel_prefill_generation_matches_sequential(cuda):
    """Greedy generation with the batched caption prefill == with the T-1 sequential decode steps."""
    torch.manual_seed(0)
    cfg = _cfg(True)
    m = DALLE(cfg).eval().to(cuda)
    text = torch.randint(2, cfg.num_text_tokens, (4, cfg.text_seq_len), device=cuda)
    tb = m.prepare_text(text)
    eng = DecodeEngine(m, 4, device=cuda)
    seq = eng.generate(tb, top_k=1, seed=3, parallel_prefill=False)
    par = eng.generate(tb, top_k=1, seed=3, parallel_prefill=True)
    assert (seq == par).float().mean().item() > 0.98


def test_vq_embed_kernel(cuda):
    vae = VQGanVAE(n_embed=64, embed_dim=32, ddconfig=dict(ch=32, out_ch=3, ch_mult=(1, 2), num_res_blocks=1,
                                                           attn_resolutions=(8,), resolution=16, z_channels=32)).to(cuda)
    codes = torch.randint(0, 64, (2, 64), device=cuda)
    z = vae.embed_codes(codes)
    ref = torch.nn.functional.one_hot(codes, 64).float() @ vae.codebook
    assert torch.allclose(z, ref.view(2, 8, 8, 32).permute(0, 3, 1, 2))
    img = vae.decode(codes)
    assert img.shape == (2, 3, 16, 16)


@pytest.mark.parametrize("mode", ["2", "0"])
def test_decode_long_full_attention_chunked(cuda, mode):
    """Full attention past 384 keys takes the chunked two-pass decode-attention path -- in mode 2 with
    the new token's q / k / v summed from the QKV slabs in its prologue: compare with the PyTorch
    decode over a 64 + 32x32 sequence."""
    torch.manual_seed(0)
    c = tiny(False)
    cfg = DALLEConfig(**{**c.to_dict(), "image_size": 256, "depth": 2, "attn_types": ["full", "axial_row"],
                          "shared_attn_ids": [0, 1], "shared_ff_ids": [0, 1]})
    assert cfg.text_seq_len + cfg.image_seq_len > 384
    m = DALLE(cfg).eval()
    B = 2
    text = torch.randint(2, cfg.num_text_tokens, (B, cfg.text_seq_len))
    img = torch.randint(0, cfg.num_image_tokens, (B, cfg.image_seq_len))
    ref = DecodeEngine(m, B, device=torch.device("cpu"), use_hip=False).teacher_forced_logits(m.prepare_text(text), img)
    mg = m.to(cuda)
    eng = DecodeEngine(mg, B, device=cuda, use_hip=True, partials=int(mode))
    assert eng.skinny and eng.qkv_partials == (mode == "2")
    out = eng.teacher_forced_logits(mg.prepare_text(text.to(cuda)), img.to(cuda)).cpu()
    rel = ((out - ref).norm() / ref.norm()).item()
    assert rel < 3e-2, rel
    assert (out.argmax(-1) == ref.argmax(-1)).float().mean().item() > 0.9


@pytest.mark.parametrize("reversible", [False, True])
def test_decode_ln_tail_matches_separate_layernorm(cuda, reversible):
    """The residual projections with the next LayerNorm + shift in their last workgroups (skinny EPI 5,
    ``ln_tail``) == the projection slabs summed by a separate decode_ln_shift launch, over whole teacher-forced
    sequences (every text / image position, both shift branches); no tail's bounded wait gave up."""
    torch.manual_seed(0)
    cfg = _cfg(reversible)
    m = DALLE(cfg).eval().to(cuda)
    B = 3
    text = torch.randint(2, cfg.num_text_tokens, (B, cfg.text_seq_len), device=cuda)
    img = torch.randint(0, cfg.num_image_tokens, (B, cfg.image_seq_len), device=cuda)
    tb = m.prepare_text(text)
    sep = DecodeEngine(m, B, device=cuda, ln_tail=False)
    tail = DecodeEngine(m, B, device=cuda, ln_tail=True)
    assert not sep.ln_tail and tail.ln_tail
    a = sep.teacher_forced_logits(tb, img)
    b = tail.teacher_forced_logits(tb, img)
    assert int(tail.ln_err.item()) == 0
    rel = ((a - b).norm() / a.norm()).item()
    assert rel < 2e-3, rel
    assert (a.argmax(-1) == b.argmax(-1)).float().mean().item() > 0.98


@pytest.mark.parametrize("B", [32, 64])
def test_decode_ln_tail_reference_width(cuda, B):
    """The same at the reference model's width (d 1024, 16 heads, FF 4096: the out-proj tail takes 2 column
    chunks per thread over 4 slabs, the FF-out tail 1 chunk over 8) and the benchmark's batch rows, two layers."""
    from dalle_amd.config import bench24

    torch.manual_seed(0)
    c = bench24()
    cfg = DALLEConfig(**{**c.to_dict(), "depth": 2, "attn_types": ["axial_row", "axial_col"], "shared_attn_ids": [0, 1],
                         "shared_ff_ids": [0, 1]})
    m = DALLE(cfg).eval().to(cuda)
    text = torch.randint(2, cfg.num_text_tokens, (B, cfg.text_seq_len), device=cuda)
    img = torch.randint(0, cfg.num_image_tokens, (B, cfg.image_seq_len), device=cuda)
    tb = m.prepare_text(text)
    out = []
    for ln_tail in (False, True):
        eng = DecodeEngine(m, B, device=cuda, ln_tail=ln_tail)
        assert eng.ln_tail == ln_tail
        out.append(eng.teacher_forced_logits(tb, img))
        if ln_tail:
            assert int(eng.ln_err.item()) == 0
    rel = ((out[0] - out[1]).norm() / out[0].norm()).item()
    assert rel < 2e-3, rel
    assert (out[0].argmax(-1) == out[1].argmax(-1)).float().mean().item() > 0.98


@pytest.mark.parametrize("mode", ["2", "0"])
def test_shared_caption_text_keys_from_row0_are_exact(cuda, mode):
    """One caption repeated over the batch (the reference's generation workload): the decode attention reads the
    text positions' K / V from row 0's cache for every row. Those rows' caches hold bitwise the same values, so the
    logits are bitwise those of the per-row reads; with distinct captions the flag stays off."""
    torch.manual_seed(0)
    cfg = _cfg(False)
    m = DALLE(cfg).eval().to(cuda)
    B = 4
    one = torch.randint(2, cfg.num_text_tokens, (1, cfg.text_seq_len), device=cuda)
    tb = m.prepare_text(one.expand(B, -1).contiguous())
    img = torch.randint(0, cfg.num_image_tokens, (B, cfg.image_seq_len), device=cuda)
    out = []
    for share in (False, True):
        eng = DecodeEngine(m, B, device=cuda, partials=int(mode))
        eng.share_text = share
        out.append(eng.teacher_forced_logits(tb, img))
        assert int(eng.text_shared.item()) == int(share)
    assert torch.equal(out[0], out[1])
    eng = DecodeEngine(m, B, device=cuda)
    distinct = m.prepare_text(torch.randint(2, cfg.num_text_tokens, (B, cfg.text_seq_len), device=cuda))
    eng.prefill(distinct)
    assert int(eng.text_shared.item()) == 0


@pytest.mark.parametrize("reversible", [False, True])
def test_repeated_caption_prefill_runs_row0_only(cuda, reversible):
    """One caption over the batch: the batched caption prefill runs for row 0 alone (the decode attention reads the
    text K / V from row 0's cache; the other rows receive the LN history the first step shifts in). Greedy
    generation matches the full-batch prefill with per-row text reads."""
    torch.manual_seed(2)
    cfg = _cfg(reversible)
    m = DALLE(cfg).eval().to(cuda)
    B = 4
    one = torch.randint(2, cfg.num_text_tokens, (1, cfg.text_seq_len), device=cuda)
    tb = m.prepare_text(one.expand(B, -1).contiguous())
    full = DecodeEngine(m, B, device=cuda)
    full.share_text = False
    ref = full.generate(tb, top_k=1, seed=3, parallel_prefill=True)
    eng = DecodeEngine(m, B, device=cuda)
    got = eng.generate(tb, top_k=1, seed=3, parallel_prefill=True)
    assert int(eng.text_shared.item()) == 1
    assert (got == ref).float().mean().item() > 0.95
    # rows 1.. never had their own text caches filled: the reads really come from row 0
    assert eng.kc[0].view(B, cfg.heads, -1, cfg.dim_head)[1:, :, : eng.T - 1].abs().sum().item() == 0.0


def test_prefill_kernels_match_torch(cuda):
    """The caption-prefill kernels (decode.hip) against the PyTorch chains they replace, fp32 references:
    LN + pushed text shift + history rows, masked row softmax to bf16, the LayerScale residual update."""
    from dalle_amd.ops.hip_ops import C

    torch.manual_seed(0)
    B, P, n, D = 3, 256, 300, 1024
    x = torch.randn(B, P, D, device=cuda) * 2 + 0.5
    w, b = torch.randn(D, device=cuda), torch.randn(D, device=cuda)
    for shift in (True, False):
        hist = torch.zeros(B, n, D, dtype=torch.bfloat16, device=cuda)
        out = torch.empty(B, P, D, dtype=torch.bfloat16, device=cuda)
        C().prefill_ln_shift_(x, w, b, hist, out, shift, 1e-5)
        y = torch.nn.functional.layer_norm(x, (D,), w, b, 1e-5)
        ref = y.clone()
        if shift:
            ref[:, 1:, : D // 2] = y[:, :-1, : D // 2]
            ref[:, 0, : D // 2] = 0
        assert (hist[:, :P].float() - y).abs().max().item() < 0.05
        assert torch.count_nonzero(hist[:, P:]) == 0  # nothing past the caption rows
        assert (out.float() - ref).abs().max().item() < 0.05
    R = 2 * 16
    sc = torch.randn(R, P, P, device=cuda) * 3
    mask = torch.tril(torch.ones(P, P, dtype=torch.bool, device=cuda))
    mask[5, :3] = False  # a non-causal hole: the kernel reads the mask, it does not assume causality
    pr = torch.empty(R, P, P, dtype=torch.bfloat16, device=cuda)
    C().prefill_softmax_(sc, mask, pr)
    ref = torch.softmax(sc.masked_fill(~mask, float("-inf")), -1)
    assert (pr.float() - ref).abs().max().item() < 4e-3
    assert torch.count_nonzero(pr.float() * (~mask).float()) == 0
    xr = torch.randn(B, P, D, device=cuda)
    yb = torch.randn(B, P, D, device=cuda).to(torch.bfloat16)
    s = torch.rand(D, device=cuda)
    want = xr + yb.float() * s
    C().prefill_residual_(xr, yb, s)
    assert torch.allclose(xr, want, rtol=1e-6, atol=1e-6)
