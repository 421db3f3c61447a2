"""Serving front-end (inference/serve.py) on CPU with the tiny model: request batching by sampling
parameters, power-of-two padded decode engines cached per shape, PNG responses over HTTP."""
import base64
import io
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "inference"))

from dalle_amd.config import DALLEConfig, tiny  # noqa: E402
from dalle_amd.data.tokenizer import HashingTokenizer  # noqa: E402
from dalle_amd.models.dalle import DALLE  # noqa: E402
from dalle_amd.models.vqgan import VQGanVAE  # noqa: E402


@pytest.fixture(scope="module")
def gen():
    from serve import BatchingGenerator

    torch.manual_seed(0)
    c = tiny(False)
    cfg = DALLEConfig(**{**c.to_dict(), "text_seq_len": 16, "image_size": 64})  # 8x8 codes: fast on CPU
    model = DALLE(cfg).eval()
    model.vae = VQGanVAE(n_embed=cfg.num_image_tokens, embed_dim=32,
                         ddconfig=dict(ch=32, out_ch=3, ch_mult=(1, 2), num_res_blocks=1, attn_resolutions=(8,),
                                       resolution=16, z_channels=32)).eval()
    g = BatchingGenerator(model, HashingTokenizer(vocab_size=cfg.num_text_tokens), "cpu", max_batch=8,
                          batch_window_ms=300)
    yield g
    g.close()


def test_batching_by_sampling_parameters(gen):
    a = gen.submit(["a red apple"], images_per_prompt=1, temperature=1.0, top_k=32)
    b = gen.submit(["the northern lights", "a cat"], images_per_prompt=1, temperature=1.0, top_k=32)
    c = gen.submit(["greedy"], images_per_prompt=2, temperature=0.0)
    ra, rb, rc = a.result(timeout=300), b.result(timeout=300), c.result(timeout=300)
    assert ra["batch_images"] == rb["batch_images"] == 3 and ra["batch_padded"] == 4
    assert rc["batch_images"] == 2 and rc["batch_padded"] == 2
    assert len(ra["images"]) == 1 and len(rb["images"]) == 2 and len(rc["images"]) == 2
    from PIL import Image

    img = np.array(Image.open(io.BytesIO(base64.b64decode(rb["images"][0]))))
    assert img.shape == (16 * 4, 16 * 4, 3) or img.ndim == 3
    # greedy decoding of the same prompt twice in one batch gives the same image
    assert rc["images"][0] == rc["images"][1]
    assert sorted(gen.engines) == [2, 4]


def test_http_endpoints(gen):
    from fastapi.testclient import TestClient
    from serve import create_app

    client = TestClient(create_app(gen))
    assert client.get("/health").json()["ok"]
    r = client.post("/generate", json={"prompts": ["hello"], "images_per_prompt": 2, "top_k": 16})
    assert r.status_code == 200 and len(r.json()["images"]) == 2
    assert client.post("/generate", json={"prompts": ["x"], "images_per_prompt": 99}).status_code == 400
    s = client.get("/stats").json()
    assert s["requests"] >= 1 and s["images"] >= 2 and s["batches"] >= 1


def test_multi_device_generator_spreads_requests():
    """--devices: one generator (model copy, engine cache, worker thread) per device, requests routed to
    the device with the fewest images in flight; two CPU "devices" stand in for a node's GPUs."""
    from fastapi.testclient import TestClient
    from serve import MultiDeviceGenerator, create_app, parse_devices

    assert parse_devices("cpu,cpu") == ["cpu", "cpu"] and parse_devices("0,3") == ["cuda:0", "cuda:3"]
    torch.manual_seed(0)
    c = tiny(False)
    cfg = DALLEConfig(**{**c.to_dict(), "text_seq_len": 16, "image_size": 64})
    model = DALLE(cfg).eval()
    g = MultiDeviceGenerator(model, HashingTokenizer(vocab_size=cfg.num_text_tokens), ["cpu", "cpu"], max_batch=4,
                             batch_window_ms=50)
    try:
        futs = [g.submit([f"prompt {i}"], images_per_prompt=2, temperature=0.0) for i in range(4)]
        res = [f.result(timeout=300) for f in futs]
        assert all(len(r["codes"]) == 2 for r in res)
        per = g.stats["per_device_images"]
        assert sum(per) == 8 and min(per) > 0, per   # both devices got work
        # greedy: the same prompt gives the same codes on either device (identical weight copies)
        a = g.gens[0].submit(["same"], 1, temperature=0.0).result(timeout=300)["codes"]
        b = g.gens[1].submit(["same"], 1, temperature=0.0).result(timeout=300)["codes"]
        assert a == b
        client = TestClient(create_app(g))
        assert client.get("/health").json()["device"] == "cpu,cpu"
        assert client.get("/stats").json()["images"] == 10
    finally:
        g.close()
