#!/usr/bin/env python3
"""Attention core forward + backward (rotary-fused) at the bench geometry under kernel schedule variants
(DALLE_AMD_ATTN_ORDER bit mask, read per call), interleaved rounds in one process, with a bitwise check of the
gradients against variant 0: python benchmarks/bench_attn_variants.py [batch] [variants, e.g. 0,4]."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.models.patterns import AttnGeometry  # noqa: E402
from dalle_amd.ops import hip_ops  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    variants = [int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "0,4").split(",")]
    T, S, H = 257, 32, 16
    n = T + S * S - 1
    geom = AttnGeometry(T, S, 5)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    qkv = (0.5 * torch.randn(B, n, 3 * H * 64, device=dev)).bfloat16().requires_grad_(True)
    g = torch.randn(B, n, H * 64, device=dev).bfloat16()
    for pattern in ("axial_row", "axial_col", "conv_like"):
        grads = {}
        for v in variants:
            os.environ["DALLE_AMD_ATTN_ORDER"] = str(v)
            qkv.grad = None
            hip_ops.attention_core(qkv, H, geom, pattern).backward(g)
            grads[v] = qkv.grad.clone()
        same = {v: bool(torch.equal(grads[v], grads[variants[0]])) for v in variants}
        times = {v: [] for v in variants}
        for _ in range(5):
            for v in variants:
                os.environ["DALLE_AMD_ATTN_ORDER"] = str(v)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(3):
                    hip_ops.attention_core(qkv, H, geom, pattern).backward(g)
                b.record()
                torch.cuda.synchronize()
                times[v].append(a.elapsed_time(b) * 1e3 / 3)
        print(json.dumps({"pattern": pattern, "B": B, "us_fwd_bwd": {v: round(statistics.median(t), 1) for v, t in times.items()},
                          "bitwise_equal_to_first": same}), flush=True)
    os.environ.pop("DALLE_AMD_ATTN_ORDER", None)


if __name__ == "__main__":
    main()
