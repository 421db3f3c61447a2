#!/usr/bin/env python3
"""Hand-written NT GEMM (csrc/kernels/gemm.hip) vs hipBLASLt (torch.mm) at the training shapes:
numerics check + median time / TFLOP/s per shape (one JSON line per shape)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops.ext import load_extension  # noqa: E402


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


def wgrad_sweep(M):
    """dW (N x K, fp32) = g^T x over M tokens: one GEMM with fp32 out (accumulate, beta=1) vs split-K
    batched GEMMs (fp32 partials) + the deterministic fold, as dalle_amd.ops.hip_ops.weight_grad runs them."""
    C = load_extension(required=True)
    dev = torch.device("cuda")
    for N, K in [(3072, 1024), (1024, 1024), (8192, 1024), (1024, 4096)]:
        g = torch.randn(M, N, device=dev).bfloat16()
        x = torch.randn(M, K, device=dev).bfloat16()
        acc = torch.zeros(N, K, device=dev)
        fl = 2 * M * N * K
        res = {"shape": f"wgrad_M{M}_N{N}_K{K}"}
        res["s1_TF"] = round(fl / timeit(lambda: torch.addmm(acc, g.t(), x, out_dtype=torch.float32, out=acc)) / 1e9)
        for s in (2, 4, 8, 16, 32):
            if M % s or M // s < 1024:
                continue

            def f(s=s):
                part = torch.bmm(g.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K), out_dtype=torch.float32)
                C.splitk_accum_(acc, part, True)
            res[f"s{s}_TF"] = round(fl / timeit(f) / 1e9)
        # the assembly TN weight-grad kernel (asm_wgrad_: token-major operands, split-K slabs + fold), every
        # split count whose K-range tiles
        ref = g.float().t() @ x.float()
        for s in (1, 2, 4, 5, 8, 16):
            if M % s or (M // s) % 128 or M // s < 256:
                continue
            out = torch.zeros(N, K, device=dev)
            C.asm_wgrad_(out, g, x, s, True)
            res[f"asm_s{s}_relerr"] = float((out - ref).norm() / ref.norm())
            res[f"asm_s{s}_TF"] = round(fl / timeit(lambda s=s: C.asm_wgrad_(acc, g, x, s, True)) / 1e9)
        print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=61440)
    ap.add_argument("--wgrad", action="store_true", help="weight-grad shapes: dW = g^T x, split-K sweep")
    args = ap.parse_args()
    if args.wgrad:
        return wgrad_sweep(args.m)
    C = load_extension(required=True)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    # correctness on a small asymmetric case first
    A = torch.randn(512, 192, device=dev).bfloat16()
    B = torch.randn(768, 192, device=dev).bfloat16()
    bias = torch.randn(768, device=dev).bfloat16()
    ref = (A.float() @ B.float().t() + bias.float())
    got = C.gemm_nt(A, B, bias).float()
    err = ((got - ref).norm() / ref.norm()).item()
    A2 = torch.randn(512, 320, device=dev).bfloat16()
    B2 = torch.randn(768, 320, device=dev).bfloat16()
    ref2 = A2.float() @ B2.float().t()
    err2 = ((C.gemm_nt(A2, B2, None, 200).float() - ref2).norm() / ref2.norm()).item()
    print(json.dumps({"check": "gemm_nt small", "rel_err": err, "phased_rel_err": err2}), flush=True)
    assert err < 1e-2 and err2 < 1e-2, (err, err2)
    M = args.m
    for N, K in [(3072, 1024), (1024, 1024), (8192, 1024), (1024, 4096), (4096, 1024)]:
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(N, K, device=dev).bfloat16()
        bias = torch.randn(N, device=dev).bfloat16()
        fl = 2 * M * N * K
        t_lt = timeit(lambda: torch.addmm(bias, A, B.t()))
        t_me = timeit(lambda: C.gemm_nt(A, B, bias))
        t_v1 = timeit(lambda: C.gemm_nt(A, B, bias, 200))
        opts = {o: round(fl / timeit(lambda: C.gemm_nt(A, B, bias, o)) / 1e9)
                for o in (202, 300, 301, 302, 308, 316, 332, 401, 402, 404, 408, 416)}
        opts["hipblaslt_again"] = round(fl / timeit(lambda: torch.addmm(bias, A, B.t())) / 1e9)
        e8 = (C.gemm_nt(A, B, bias, 300).float() - torch.addmm(bias, A, B.t()).float()).abs().max().item()
        e2 = ((C.gemm_nt(A, B, bias, 200).float() - torch.addmm(bias, A, B.t()).float()).norm() /
              torch.addmm(bias, A, B.t()).float().norm()).item()
        e = ((C.gemm_nt(A, B, bias).float() - torch.addmm(bias, A, B.t()).float()).norm() /
             torch.addmm(bias, A, B.t()).float().norm()).item()
        print(json.dumps({"shape": f"M{M}_N{N}_K{K}", "hipblaslt_TF": round(fl / t_lt / 1e9), "ours_TF": round(fl / t_me / 1e9), "ours_phased_TF": round(fl / t_v1 / 1e9), "phased_err": e2, "8ph_maxdiff": e8, "opts_TF": opts,
                          "hipblaslt_ms": round(t_lt, 4), "ours_ms": round(t_me, 4), "rel_err_vs_hipblaslt": e}), flush=True)


if __name__ == "__main__":
    main()
