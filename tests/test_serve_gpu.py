"""Serving front-end on MI355X: batches run through hipGraph-captured decode engines (one per padded
batch shape, replayed for later batches) and the fused sampler."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "inference"))

from dalle_amd.config import DALLEConfig, tiny  # noqa: E402
from dalle_amd.data.tokenizer import HashingTokenizer  # noqa: E402
from dalle_amd.models.dalle import DALLE  # noqa: E402
from dalle_amd.models.vqgan import VQGanVAE  # noqa: E402

pytestmark = pytest.mark.gpu


def test_serving_on_gpu(cuda):
    from serve import BatchingGenerator

    torch.manual_seed(0)
    cfg = tiny(False)
    model = DALLE(cfg).eval()
    model.vae = VQGanVAE(n_embed=cfg.num_image_tokens, embed_dim=32,
                         ddconfig=dict(ch=32, out_ch=3, ch_mult=(1, 2), num_res_blocks=1, attn_resolutions=(16,),
                                       resolution=32, z_channels=32)).eval()
    model = model.to(cuda)
    gen = BatchingGenerator(model, HashingTokenizer(vocab_size=cfg.num_text_tokens), cuda, max_batch=16,
                            batch_window_ms=200)
    try:
        futs = [gen.submit([f"prompt {i}"], images_per_prompt=2, temperature=1.0, top_k=64) for i in range(3)]
        res = [f.result(timeout=100) for f in futs]
        assert all(r["batch_images"] == 6 and r["batch_padded"] == 8 for r in res)
        assert all(len(r["images"]) == 2 for r in res)
        assert gen.engines[8].graph is not None  # the decode step was captured
        again = gen.submit(["prompt 0"], images_per_prompt=8, temperature=0.0).result(timeout=100)
        assert again["batch_padded"] == 8
        # greedy: the same codes 8 times; the VQGAN decode of a batch may differ by ~1e-6 per image, so
        # compare pixels with one 8-bit level of slack instead of the PNG bytes
        import base64
        import io

        import numpy as np
        from PIL import Image

        px = [np.asarray(Image.open(io.BytesIO(base64.b64decode(b)))).astype(int) for b in again["images"]]
        assert all(np.abs(a - px[0]).max() <= 1 for a in px)
    finally:
        gen.close()


def test_multi_device_serving_concurrent_captures(cuda):
    """Two generators (model copies, engine caches, worker threads) share the GPU here, standing in for a
    node's devices: their first batches capture hipGraphs while the other thread replays -- captures run
    one at a time in thread-local mode -- and greedy results match across the copies."""
    from serve import MultiDeviceGenerator

    torch.manual_seed(0)
    cfg = tiny(False)
    model = DALLE(cfg).eval()
    dev = str(cuda)
    g = MultiDeviceGenerator(model, HashingTokenizer(vocab_size=cfg.num_text_tokens), [dev, dev], max_batch=8,
                             batch_window_ms=20)
    try:
        futs = [g.submit([f"p{i}"], images_per_prompt=[1, 2, 4, 8][i % 4], temperature=1.0, top_k=32) for i in range(12)]
        res = [f.result(timeout=100) for f in futs]
        assert sum(len(r["codes"]) for r in res) == 3 * (1 + 2 + 4 + 8)
        assert min(g.stats["per_device_images"]) > 0
        a = g.gens[0].submit(["same"], 4, temperature=0.0).result(timeout=100)["codes"]
        b = g.gens[1].submit(["same"], 4, temperature=0.0).result(timeout=100)["codes"]
        assert a == b
    finally:
        g.close()
