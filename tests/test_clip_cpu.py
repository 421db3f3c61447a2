"""Native CLIP ViT-B/32 re-ranker: architecture / key layout, preprocessing, scores."""
import torch

from dalle_amd.models.clip import CLIP, ClipConfig, ClipTokenizer, clip_scores, load_clip, preprocess


def _small():
    return ClipConfig(embed_dim=32, image_resolution=64, vision_layers=2, vision_width=64, vision_patch_size=32,
                      context_length=16, vocab_size=49408, transformer_width=32, transformer_heads=2, transformer_layers=2)


def test_openai_key_layout_and_param_count():
    m = CLIP()
    keys = set(m.state_dict().keys())
    for k in ["visual.conv1.weight", "visual.class_embedding", "visual.positional_embedding", "visual.proj",
              "visual.transformer.resblocks.11.attn.in_proj_weight", "visual.transformer.resblocks.0.mlp.c_fc.weight",
              "transformer.resblocks.11.attn.out_proj.weight", "token_embedding.weight", "positional_embedding",
              "ln_final.weight", "text_projection", "logit_scale"]:
        assert k in keys, k
    n = sum(p.numel() for p in m.parameters())
    assert abs(n - 151_277_313) < 1_000  # ViT-B/32 CLIP parameter count


def test_scores_and_roundtrip(tmp_path):
    torch.manual_seed(0)
    m = CLIP(_small()).eval()
    tok = ClipTokenizer(context_length=16)
    t = tok(["a red apple", "a cat"])
    assert t[0, 0] == ClipTokenizer.SOT and (t[0] == ClipTokenizer.EOT).sum() == 1
    imgs = torch.rand(5, 80, 96, 3)
    x = preprocess(imgs, resolution=64)
    assert x.shape == (5, 3, 64, 64)
    with torch.no_grad():
        li, lt = m(x, t)
    assert li.shape == (5, 2) and torch.allclose(li.t(), lt)
    path = tmp_path / "clip.pt"
    torch.save(m.state_dict(), path)
    m2 = CLIP(_small())
    m2.load_state_dict(torch.load(path, weights_only=True))
    img = preprocess(imgs, 64)
    s1 = torch.softmax(m(img, t[:1])[1][0], -1)
    s2 = torch.softmax(m2.eval()(img, t[:1])[1][0], -1)
    assert torch.allclose(s1, s2) and abs(float(s1.sum()) - 1) < 1e-5


def test_clip_scores_full_size_random():
    m = load_clip(None)
    s = clip_scores(m, ClipTokenizer(), torch.rand(3, 256, 256, 3), "a painting of a fox")
    assert s.shape == (3,) and abs(float(s.sum()) - 1) < 1e-4
