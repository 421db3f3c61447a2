#!/usr/bin/env python3
"""Attention core fwd + bwd (rotary-fused backward) at the bench geometry, repeated, for counter
collection: python benchmarks/bench_attn_kernel.py [pattern] [batch] [reps]."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.models.patterns import AttnGeometry  # noqa: E402
from dalle_amd.ops import hip_ops  # noqa: E402


def main():
    pattern = sys.argv[1] if len(sys.argv) > 1 else "axial_row"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    T, S, H = 257, 32, 16
    n = T + S * S - 1
    geom = AttnGeometry(T, S, 5)
    dev = torch.device("cuda")
    qkv = torch.randn(B, n, 3 * H * 64, device=dev).bfloat16().requires_grad_(True)
    g = torch.randn(B, n, H * 64, device=dev).bfloat16()
    for _ in range(2):
        hip_ops.attention_core(qkv, H, geom, pattern).backward(g)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        hip_ops.attention_core(qkv, H, geom, pattern).backward(g)
    torch.cuda.synchronize()
    print(f"{pattern} B={B}: {(time.perf_counter() - t) / reps * 1e3:.3f} ms per fwd+bwd")


if __name__ == "__main__":
    main()
