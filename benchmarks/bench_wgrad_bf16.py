#!/usr/bin/env python3
"""Weight-gradient GEMM: fp32-output partials (production, hipBLASLt BSS kernels) against bf16-output
partials (the tuned BBS kernels the forward / input-gradient GEMMs run on) at the training shapes
(M = 61440 tokens, bench24 micro-batch 48). Times the split-K GEMM alone and GEMM + fold (TF/s).

    python benchmarks/bench_wgrad_bf16.py
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
        fl = 2.0 * M * N * K
        for s in (1, 2, 4, 8, 16):
            res = {"shape": f"N{N}_K{K}_M{M}", "split": s}
            gv, xv = g.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K)
            res["fp32_gemm_TF"] = round(fl / timeit(lambda: torch.bmm(gv, xv, out_dtype=torch.float32)) / 1e9)
            res["bf16_gemm_TF"] = round(fl / timeit(lambda: torch.bmm(gv, xv)) / 1e9)
            # the same product with the operands swapped (x^T g): the transposed problem
            xt, gt = x.view(s, M // s, K).transpose(1, 2), g.view(s, M // s, N)
            res["bf16_gemm_T_TF"] = round(fl / timeit(lambda: torch.bmm(xt, gt)) / 1e9)
            if s > 1:
                res["fp32_full_TF"] = round(fl / timeit(lambda: C.splitk_accum_(out, torch.bmm(gv, xv, out_dtype=torch.float32), True)) / 1e9)
                res["bf16_full_TF"] = round(fl / timeit(lambda: out.add_(torch.bmm(gv, xv).sum(0, dtype=torch.float32))) / 1e9)
            print(json.dumps(res), flush=True)
        del g, x, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
