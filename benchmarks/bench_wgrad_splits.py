#!/usr/bin/env python3
"""Weight-gradient GEMM split-K sweep at the training shapes (M = 61440 tokens, bench24 micro-batch 48):
dW (N, K) fp32 = sum over s token slices of dY_s^T X_s, as the production path runs it (hipBLASLt batched
GEMM with fp32 partials + the deterministic fold kernel, hip_ops.weight_grad). Prints TF/s per split.

    python benchmarks/bench_wgrad_splits.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops.ext import load_extension  # noqa: E402


def timeit(fn, reps=10, warmup=3):
    for _ in range(warmup):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    C = load_extension(required=True)
    dev = torch.device("cuda")
    M = int(os.environ.get("M", 61440))
    for N, K in [(1024, 1024), (3072, 1024), (1024, 4096), (8192, 1024)]:
        g = torch.randn(M, N, device=dev).bfloat16()
        x = torch.randn(M, K, device=dev).bfloat16()
        out = torch.zeros(N, K, device=dev)
        res = {"shape": f"N{N}_K{K}_M{M}"}
        for s in (1, 2, 3, 4, 6, 8, 12, 16, 24):
            if M % s:
                continue
            if s == 1:
                fn = lambda: torch.addmm(out, g.t(), x, out_dtype=torch.float32, out=out)  # noqa: E731
            else:
                def fn(s=s):
                    part = torch.bmm(g.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K), out_dtype=torch.float32)
                    C.splitk_accum_(out, part, True)
            res[f"s{s}"] = round(2.0 * M * N * K / timeit(fn) / 1e9)
        print(json.dumps(res), flush=True)
        del g, x, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
