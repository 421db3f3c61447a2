#!/usr/bin/env python3
"""Batched caption prefill of the decode engine (reference model, batch 64, distinct captions; SAME=1: one caption
repeated over the batch): wall time per call."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.config import get_config  # noqa: E402
from dalle_amd.models.dalle import DALLE  # noqa: E402
from dalle_amd.models.generation import make_decode_engine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config(os.environ.get("MODEL", "reference"))
    model = DALLE(cfg).to(dev).eval()
    B = int(os.environ.get("BATCH", 64))
    rows = 1 if os.environ.get("SAME") == "1" else B
    text = torch.randint(2, cfg.num_text_tokens, (rows, cfg.text_seq_len), device=dev).expand(B, -1).contiguous()
    eng = make_decode_engine(model, B, device=dev)  # the split engine at batch >= 32, as generate_images uses
    tb = model.prepare_text(text)
    for _ in range(2):
        eng.prefill_parallel(tb)
    torch.cuda.synchronize()
    t = time.perf_counter()
    reps = 3
    for _ in range(reps):
        eng.prefill_parallel(tb)
    torch.cuda.synchronize()
    print(f'{{"prefill_ms": {(time.perf_counter() - t) / reps * 1e3:.1f}, "batch": {B}, "positions": {cfg.text_len - 1}}}', flush=True)


if __name__ == "__main__":
    main()
