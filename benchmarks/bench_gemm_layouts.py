#!/usr/bin/env python3
"""hipBLASLt at the training step's activation GEMMs: C (M, N) = A (M, K) . B (K, N) with each operand
stored row-major or transposed (4 storage combinations of the same product), to see whether a different
operand layout makes the library pick a faster solution. M = 61440 tokens (bench24, micro-batch 48).

    python benchmarks/bench_gemm_layouts.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=20, warmup=3):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def wgrad(M, dev):
    """dW (N_out, K_in) fp32 = dY^T X over M tokens, each operand stored either way (the contraction runs
    over the tokens): which storage makes the weight-gradient GEMMs fastest."""
    for N, K in [(3072, 1024), (1024, 1024), (8192, 1024), (1024, 4096)]:
        g = torch.randn(M, N, device=dev).bfloat16()
        x = torch.randn(M, K, device=dev).bfloat16()
        gt, xt = g.t().contiguous(), x.t().contiguous()
        out = torch.empty(N, K, device=dev, dtype=torch.float32)
        fl = 2.0 * M * N * K
        res = {"shape": f"wgrad_N{N}_K{K}_M{M}"}
        # A = dY^T (N x M): a transposed view of g (cm) or gt (rm); B = X (M x K): x (rm) or xt.t() (cm)
        for an, a in (("A_rm", gt), ("A_cm", g.t())):
            for bn, b in (("B_rm", x), ("B_cm", xt.t())):
                res[f"{an}_{bn}_TF"] = round(fl / timeit(lambda: torch.mm(a, b, out_dtype=torch.float32, out=out)) / 1e9)
        print(json.dumps(res), flush=True)
        del g, x, gt, xt, out
        torch.cuda.empty_cache()


def main():
    M = int(os.environ.get("M", 61440))
    if "--wgrad" in sys.argv:
        return wgrad(M, torch.device("cuda"))
    dev = torch.device("cuda")
    torch.manual_seed(0)
    # forward (x . W^T): (N, K) = (3072, 1024) QKV, (1024, 1024) out-proj, (8192, 1024) FF-in, (1024, 4096) FF-out;
    # input gradients (dy . W): (1024, 3072) QKV, (1024, 8192) FF-in
    shapes = [(3072, 1024), (1024, 1024), (8192, 1024), (1024, 4096), (1024, 3072), (1024, 8192)]
    for N, K in shapes:
        a_rm = torch.randn(M, K, device=dev).bfloat16()
        b_rm = torch.randn(K, N, device=dev).bfloat16()
        a_cm = a_rm.t().contiguous().t()  # same values, column-major storage
        b_cm = b_rm.t().contiguous().t()
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        res = {"shape": f"M{M}_N{N}_K{K}"}
        ref = None
        for an, a in (("A_rm", a_rm), ("A_cm", a_cm)):
            for bn, b in (("B_rm", b_rm), ("B_cm", b_cm)):
                torch.mm(a, b, out=out)
                if ref is None:
                    ref = out.float().clone()
                else:
                    assert torch.allclose(out.float(), ref, rtol=2e-2, atol=1e-1)
                res[f"{an}_{bn}_TF"] = round(fl / timeit(lambda: torch.mm(a, b, out=out)) / 1e9)
        print(json.dumps(res), flush=True)
        del a_rm, b_rm, a_cm, b_cm, out, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
