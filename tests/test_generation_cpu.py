"""KV-cache decoding == full forward (static masks, cached token shift, rotary at position)."""
import os

import pytest
import torch

from dalle_amd.config import DALLEConfig, tiny
from dalle_amd.models.dalle import DALLE
from dalle_amd.models.generation import DecodeEngine, filter_logits
from dalle_amd.models.vqgan import VQGanVAE


def _cfg(reversible):
    c = tiny(reversible)
    return DALLEConfig(**{**c.to_dict(), "depth": 4, "attn_types": ["axial_row", "axial_col", "conv_like", "full"],
                          "shared_attn_ids": [0, 1, 2, 3], "shared_ff_ids": [0, 1, 0, 1]})


@pytest.mark.parametrize("reversible", [False, True])
def test_teacher_forced_decode_matches_forward(reversible):
    torch.manual_seed(0)
    cfg = _cfg(reversible)
    m = DALLE(cfg).eval()
    B = 2
    text = torch.randint(2, cfg.num_text_tokens, (B, cfg.text_seq_len))
    text[:, 30:] = 1
    img = torch.randint(0, cfg.num_image_tokens, (B, cfg.image_seq_len))
    with torch.no_grad():
        full = m(text, img, return_loss=False)  # (B, n, V) masked logits
    eng = DecodeEngine(m, B, device=torch.device("cpu"), use_hip=False)
    dec = eng.teacher_forced_logits(m.prepare_text(text), img)  # (B, 256, V_img)
    ref = full[:, cfg.text_seq_len:, m.num_text_tokens:]
    assert dec.shape == ref.shape
    assert torch.allclose(dec, ref, atol=2e-4, rtol=1e-4), (dec - ref).abs().max()


def test_generate_images_and_filters():
    torch.manual_seed(0)
    cfg = _cfg(False)
    m = DALLE(cfg).eval()
    text = torch.randint(2, cfg.num_text_tokens, (3, cfg.text_seq_len))
    codes = m.generate_images(text, top_k=16, top_p=0.9, temperature=0.7)
    assert codes.shape == (3, cfg.image_seq_len)
    assert codes.min() >= 0 and codes.max() < cfg.num_image_tokens
    logits = torch.randn(4, 100)
    f = filter_logits(logits, top_k=5)
    assert (torch.isfinite(f).sum(-1) == 5).all()
    f = filter_logits(logits, top_p=0.5)
    assert (torch.isfinite(f).sum(-1) >= 1).all()


def test_vqgan_decode_shapes():
    torch.manual_seed(0)
    vae = VQGanVAE(n_embed=64, embed_dim=32, ddconfig=dict(ch=32, out_ch=3, ch_mult=(1, 2), num_res_blocks=1,
                                                           attn_resolutions=(8,), resolution=16, z_channels=32))
    codes = torch.randint(0, 64, (2, 64))
    img = vae.decode(codes)
    assert img.shape == (2, 3, 16, 16) and img.min() >= 0 and img.max() <= 1
    z = vae.embed_codes(codes)
    one_hot = torch.nn.functional.one_hot(codes, 64).float() @ vae.codebook
    assert torch.allclose(z, one_hot.view(2, 8, 8, 32).permute(0, 3, 1, 2))


_SMALL_DD = dict(ch=32, out_ch=3, ch_mult=(1, 2), num_res_blocks=1, attn_resolutions=(8,), resolution=16, z_channels=32)


def test_vqgan_encoder_codes():
    """get_codebook_indices (dalle-pytorch API): gumbel = argmax of the proj logits, plain VQ = nearest
    codebook vector; taming checkpoint naming (incl. ``quantize.embedding``) loads; a decoder-only
    checkpoint still decodes but refuses to encode."""
    torch.manual_seed(0)
    img = torch.rand(2, 3, 16, 16)
    g = VQGanVAE(n_embed=64, embed_dim=32, ddconfig=_SMALL_DD, is_gumbel=True)
    idx = g.get_codebook_indices(img)
    assert idx.shape == (2, 64) and idx.dtype == torch.int64 and 0 <= idx.min() and idx.max() < 64
    h = g.quant_conv(g.encoder(2 * img - 1))
    assert torch.equal(idx, g.quantize.proj(h).argmax(1).flatten(1))
    assert torch.equal(idx, g.get_codebook_indices(img))  # the mode is deterministic
    s = g.get_codebook_indices(img, gumbel_tau=1.0, generator=torch.Generator().manual_seed(1))
    assert s.shape == idx.shape
    assert g.decode(idx).shape == (2, 3, 16, 16)

    v = VQGanVAE(n_embed=64, embed_dim=32, ddconfig=_SMALL_DD, is_gumbel=False)
    assert v.quantize.proj is None
    vi = v.get_codebook_indices(img)
    z = v.quant_conv(v.encoder(2 * img - 1)).permute(0, 2, 3, 1).reshape(-1, 32)
    assert torch.equal(vi.flatten(), torch.cdist(z, v.codebook).argmin(1))


def test_vqgan_checkpoint_naming(tmp_path):
    torch.manual_seed(0)
    src = VQGanVAE(n_embed=64, embed_dim=32, ddconfig=_SMALL_DD, is_gumbel=False)
    sd = src.state_dict()
    sd["quantize.embedding.weight"] = sd.pop("quantize.embed.weight")  # taming VectorQuantizer name
    import yaml

    cfg = tmp_path / "vq.yaml"
    cfg.write_text(yaml.safe_dump({"model": {"target": "taming.models.vqgan.VQModel", "params": {
        "n_embed": 64, "embed_dim": 32, "ddconfig": {**_SMALL_DD, "ch_mult": [1, 2], "attn_resolutions": [8]}}}}))
    torch.save({"state_dict": sd}, tmp_path / "full.ckpt")
    full = VQGanVAE(str(tmp_path / "full.ckpt"), str(cfg))
    img = torch.rand(1, 3, 16, 16)
    assert torch.equal(full.get_codebook_indices(img), src.get_codebook_indices(img))
    dec_only = {k: v for k, v in sd.items() if not k.startswith(("encoder.", "quant_conv."))}
    torch.save({"state_dict": dec_only}, tmp_path / "dec.ckpt")
    d = VQGanVAE(str(tmp_path / "dec.ckpt"), str(cfg))
    codes = torch.randint(0, 64, (1, 64))
    assert torch.allclose(d.decode(codes), src.decode(codes))
    with pytest.raises(RuntimeError):
        d.get_codebook_indices(img)


@pytest.mark.parametrize("reversible", [False, True])
def test_parallel_prefill_matches_sequential_steps(reversible):
    """The batched caption prefill fills the KV caches and LN histories as the T-1 decode steps do and
    leaves the engine at the same position: the next step's logits agree."""
    torch.manual_seed(0)
    cfg = _cfg(reversible)
    m = DALLE(cfg).eval()
    B = 3
    text = torch.randint(2, cfg.num_text_tokens, (B, cfg.text_seq_len))
    text[:, 40:] = 0  # padding -> the unique per-position pad ids
    tb = m.prepare_text(text)
    seq = DecodeEngine(m, B, device=torch.device("cpu"), use_hip=False)
    par = DecodeEngine(m, B, device=torch.device("cpu"), use_hip=False)
    with torch.no_grad():
        seq.prefill(tb)
        par.prefill_parallel(tb)
        P = cfg.text_len - 1
        assert int(seq.pos) == int(par.pos) == P and torch.equal(seq.tok, par.tok)
        for li in range(len(seq.kc)):
            for a, b in ((seq.kc[li], par.kc[li]), (seq.vc[li], par.vc[li])):
                assert torch.allclose(a[:, :P], b[:, :P], atol=1e-4, rtol=1e-4)
                assert not b[:, P:].any()
            for j in range(2):
                assert torch.allclose(seq.hist[li][j][:, :P], par.hist[li][j][:, :P], atol=1e-4, rtol=1e-4)
        l_seq, l_par = seq._forward_position(), par._forward_position()
    assert torch.allclose(l_seq, l_par, atol=2e-4, rtol=1e-4), (l_seq - l_par).abs().max()


def test_run_inference_spreads_queries_over_devices(tmp_path):
    """inference/run_inference.py --devices: one model copy per device, queries taken by per-device workers;
    every query gets its pickle (reference output format: query, temperature, images, clip_scores)."""
    import pickle
    import subprocess
    import sys as _sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    (tmp_path / "q.txt").write_text("a red apple\nthe northern lights\n\na cat\n")
    r = subprocess.run([_sys.executable, os.path.join(root, "inference", "run_inference.py"), "--queries", str(tmp_path / "q.txt"),
                        "--model-preset", "tiny", "--output-dir", str(tmp_path / "out"), "--batch-size", "1", "--n-iters", "2",
                        "--devices", "cpu,cpu", "--top-k", "16"], capture_output=True, text=True, timeout=600,
                       env={k: v for k, v in os.environ.items() if k != "HIP_VISIBLE_DEVICES"} | {"HIP_VISIBLE_DEVICES": ""})
    assert r.returncode == 0, r.stderr[-3000:]
    assert "2 devices" in r.stdout
    for q in ("a red apple", "the northern lights", "a cat"):
        with open(tmp_path / "out" / f"{q}.pickle", "rb") as f:  # written by this test's own subprocess
            out = pickle.load(f)
        assert out["query"] == q and len(out["images"]) == 2 and out["clip_scores"].shape == (2,)
