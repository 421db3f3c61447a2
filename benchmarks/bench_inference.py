#!/usr/bin/env python3
"""BASELINE config 5: text->image top-k sampling, batch 64 on one MI355X, hipGraph-replayed decode.

Reference model recipe (64 layers, 5 shared blocks, reversible) with random-init weights and a
random-init VQGAN decoder; prints one JSON line with images/s (end-to-end: prefill + 1024 decode
steps + VQGAN decode) and the per-token decode latency.
"""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--model", default="reference")
    ap.add_argument("--top-k", type=int, default=256)
    ap.add_argument("--iters", type=int, default=2)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-vae", action="store_true")
    ap.add_argument("--same-caption", action="store_true",
                    help="one caption repeated over the batch, as inference/run_inference.py generates (the decode "
                         "attention then reads the text keys from one cache row); default: a distinct caption per row")
    ap.add_argument("--profile-steps", type=int, default=0,
                    help="batched caption prefill + N image-position decode steps (graph replays unless --no-graph), "
                         "then exit (rocprof)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    cfg = get_config(args.model)
    model = DALLE(cfg).to(dev).eval()
    if not args.no_vae:
        model.vae = VQGanVAE().to(dev).eval()
    text = torch.randint(2, cfg.num_text_tokens, (1 if args.same_caption else args.batch, cfg.text_seq_len), device=dev)
    text = text.expand(args.batch, -1).contiguous()
    use_graph = not args.no_graph
    from dalle_amd.models.generation import make_decode_engine
    eng = make_decode_engine(model, args.batch, device=dev)
    model._decode_engine = eng
    parts = getattr(eng, "nparts", 1)
    tb = model.prepare_text(text)
    prefill = getattr(eng, "prefill_parallel", eng.prefill)
    # warm-up generate (captures the step graph)
    t = time.perf_counter()
    model.generate_images(text, top_k=args.top_k, use_graph=use_graph)
    torch.cuda.synchronize()
    print(f"# warm-up generate done: {time.perf_counter() - t:.2f}s", file=sys.stderr, flush=True)
    t = time.perf_counter()
    prefill(tb)
    torch.cuda.synchronize()
    print(f"# batched prefill of {cfg.text_len} caption positions: {(time.perf_counter() - t) * 1e3:.1f} ms", file=sys.stderr,
          flush=True)
    if args.profile_steps:
        # image positions only (the text-key part of every sparse pattern is read from here on)
        if use_graph and hasattr(eng, "replay_steps"):
            eng.replay_steps(args.profile_steps)
        for _ in range(0 if (use_graph and hasattr(eng, "replay_steps")) else args.profile_steps):
            eng.graph.replay() if use_graph else eng._image_step()
        torch.cuda.synchronize()
        return
    # one more untimed generate: the first one after the standalone prefill above runs ~0.3 s slow
    # (profiles/r3_decode_partials_cols.txt), which is not the steady-state rate
    model.generate_images(text, top_k=args.top_k, use_graph=use_graph)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.iters):
        out = model.generate_images(text, top_k=args.top_k, use_graph=use_graph)
        torch.cuda.synchronize()
        print(f"# generate {i}: {time.perf_counter() - t0:.2f}s", file=sys.stderr, flush=True)
    el = (time.perf_counter() - t0) / args.iters
    # sampling alone (no VAE): batched caption prefill + 1024 decode steps, per sampled image token
    t2 = time.perf_counter()
    model.generate_images(text, top_k=args.top_k, use_graph=use_graph, return_codes=True)
    torch.cuda.synchronize()
    codes_s = time.perf_counter() - t2
    eng = model._decode_engine
    # decode-only timing: 256 image positions right after the batched caption prefill (every step
    # reads the 256 text keys of each layer's cache plus its local image keys). 256, not 64: the two
    # chains' per-part graphs run free and the window ends on the later one (~19 ms per window,
    # profiles/r6_decode_replay_host.txt), which a 64-step window would spread as +0.3 ms per step
    NDEC = 256
    prefill(tb)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if use_graph and hasattr(eng, "replay_steps"):
        eng.replay_steps(NDEC)
    for _ in range(0 if (use_graph and hasattr(eng, "replay_steps")) else NDEC):
        eng.graph.replay() if use_graph else eng._step()
    torch.cuda.synchronize()
    per_tok = (time.perf_counter() - t1) / NDEC
    print(json.dumps({"metric": "text->image generation throughput (batch 64, top-k, hipGraph decode)",
                      "value": round(args.batch / el, 3), "unit": "images/s", "n_gpus": 1,
                      "seconds_per_batch": round(el, 3), "ms_per_decode_step": round(per_tok * 1e3, 3),
                      "decode_step_positions": f"image positions {cfg.text_len - 1}..{cfg.text_len + NDEC - 2}",
                      "ms_per_image_token": round(codes_s / cfg.image_seq_len * 1e3, 3),
                      "sampling_seconds": round(codes_s, 3), "decode_parts": parts,
                      "batch": args.batch, "model": args.model, "depth": cfg.depth, "graph": use_graph,
                      "vae": not args.no_vae, "out_shape": list(out.shape), "dtype": "bf16",
                      "captions": "one repeated" if args.same_caption else "distinct per row",
                      "text_shared": [int(e.text_shared.item()) for e in getattr(eng, "parts", [eng])],
                      "data": "random-init weights, synthetic captions"}), flush=True)


if __name__ == "__main__":
    main()
