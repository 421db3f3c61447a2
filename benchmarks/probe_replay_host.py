#!/usr/bin/env python3
"""Host side of the hipGraph decode replay: how long does the CPU take to submit one image-position step
(graph.replay(), no synchronisation) against how long the GPU takes to run it? If submission is not far
ahead of execution, host jitter shows up as GPU idle time between kernels.

Reference model, batch 64, repeated caption; prints one JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dalle_amd.config import get_config  # noqa: E402
from dalle_amd.models.dalle import DALLE  # noqa: E402
from dalle_amd.models.generation import DecodeEngine, SplitDecodeEngine, make_decode_engine  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config(os.environ.get("PROBE_MODEL", "reference"))
    B = int(os.environ.get("PROBE_BATCH", "64"))
    model = DALLE(cfg).to(dev).eval()
    text = torch.randint(2, cfg.num_text_tokens, (1, cfg.text_seq_len), device=dev).expand(B, -1).contiguous()
    parts = int(os.environ.get("PROBE_PARTS", "0"))
    if parts == 1:
        eng = DecodeEngine(model, B, device=dev)
    elif parts > 1:
        eng = SplitDecodeEngine(model, B, device=dev, parts=parts)
    else:
        eng = make_decode_engine(model, B, device=dev)
    model._decode_engine = eng
    model.generate_images(text, top_k=256, use_graph=True, return_codes=True)
    torch.cuda.synchronize()
    tb = model.prepare_text(text)
    res = {}
    # k steps: replay_steps (a split engine forks its part streams once and joins them at the end)
    replay = eng.replay_steps if hasattr(eng, "replay_steps") else (lambda k: [eng.graph.replay() for _ in range(k)])
    # submission cost with an EMPTY queue: one / two / four replays right after a synchronize
    for n in (1, 2, 4):
        eng.prefill_parallel(tb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        replay(n)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        res[f"empty_queue_{n}"] = round((t1 - t0) / n * 1e3, 3)
    for n in (16, 64, 256):
        eng.prefill_parallel(tb)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        replay(n)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res[n] = {"host_submit_ms_per_step": round((t1 - t0) / n * 1e3, 3),
                  "wall_ms_per_step": round((t2 - t0) / n * 1e3, 3)}
        print(f"# {n} replays: submit {res[n]['host_submit_ms_per_step']} ms/step, wall {res[n]['wall_ms_per_step']} ms/step",
              file=sys.stderr, flush=True)
    # the same 64 steps between events on the current stream (a split engine joins its part streams there)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    eng.prefill_parallel(tb)
    torch.cuda.synchronize()
    ev0.record()
    replay(64)
    ev1.record()
    torch.cuda.synchronize()
    res["event_ms_per_step"] = round(ev0.elapsed_time(ev1) / 64, 3)
    # the step time along the image: 16 chunks of 64 positions after one prefill
    chunks = []
    eng.prefill_parallel(tb)
    torch.cuda.synchronize()
    for _ in range(cfg.image_seq_len // 64):
        t0 = time.perf_counter()
        replay(64)
        torch.cuda.synchronize()
        chunks.append(round((time.perf_counter() - t0) / 64 * 1e3, 3))
    res["ms_per_step_by_64_positions"] = chunks
    env = {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_", "PROBE_", "DALLE_AMD_"))}
    print(json.dumps({"probe": "decode graph replay, host submit vs GPU", "batch": B, "model": cfg.depth, "env": env,
                      "parts": getattr(eng, "nparts", 1),
                      "graphs": getattr(eng, "graph_mode", "linear"), "results": res}), flush=True)


if __name__ == "__main__":
    main()
