#!/usr/bin/env python3
"""Where generate_images' time goes outside the decode steps: interleaved timings of generate with and
without the VQGAN decode, and the VAE decode alone on the generated codes (reference model, batch 64)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.config import get_config  # noqa: E402
from dalle_amd.models.dalle import DALLE  # noqa: E402
from dalle_amd.models.vqgan import VQGanVAE  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    cfg = get_config(sys.argv[1] if len(sys.argv) > 1 else "reference")
    model = DALLE(cfg).to(dev).eval()
    model.vae = VQGanVAE().to(dev).eval()
    text = torch.randint(2, cfg.num_text_tokens, (64, cfg.text_seq_len), device=dev)
    model.generate_images(text, top_k=256)
    torch.cuda.synchronize()
    res = {"codes_s": [], "images_s": [], "vae_s": []}
    for _ in range(2):
        for kind in ("codes_s", "images_s"):
            t = time.perf_counter()
            out = model.generate_images(text, top_k=256, return_codes=(kind == "codes_s"))
            torch.cuda.synchronize()
            res[kind].append(round(time.perf_counter() - t, 3))
            if kind == "codes_s":
                codes = out
        t = time.perf_counter()
        model.vae.decode(codes)
        torch.cuda.synchronize()
        res["vae_s"].append(round(time.perf_counter() - t, 3))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
