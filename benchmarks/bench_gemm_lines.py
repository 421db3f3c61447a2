#!/usr/bin/env python3
"""Whole-line epilogue stores (round 4): the register-epilogue GEMM family (csrc/kernels/gemm_pt.hip) with
16 rows x 64 B per store instruction (lines 0, rounds 1-3) vs 8 rows x 128 B (lines 1, lines16), one tile
per workgroup and persistent, against hipBLASLt and the main loop alone, at the bench24 micro-batch-128
shapes (M = 163840 tokens; env M overrides). Random operands, interleaved rounds in one process (median).
One JSON line per shape / fused op."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops import hip_ops  # noqa: E402
from dalle_amd.models.patterns import AttnGeometry  # noqa: E402


def run(variants, rounds=5, reps=3):
    for fn in variants.values():
        fn()
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for k, fn in variants.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                fn()
            b.record()
            torch.cuda.synchronize()
            res[k].append(a.elapsed_time(b) * 1e3 / reps)
    return {k: round(statistics.median(v), 1) for k, v in res.items()}


def main():
    C = hip_ops.C()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M = int(os.environ.get("M", 163840))

    def L(lines, fn):
        def f():
            C.gemm_set_lines(lines)
            return fn()
        return f

    only = os.environ.get("ONLY", "")
    shapes = [(3072, 1024), (1024, 1024), (8192, 1024), (4096, 1024), (1024, 4096), (1024, 8192), (1024, 3072)]
    if only and only != "plain":
        shapes = []
    for N, K in shapes:
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(N, K, device=dev).bfloat16()
        v = {"hipblaslt": lambda: torch.mm(A, B.t()),
             "np_l0": L(0, lambda: C.gemm_pt(A, B, None, 30, 0)), "np_l1": L(1, lambda: C.gemm_pt(A, B, None, 30, 0)),
             "ps_l0": L(0, lambda: C.gemm_pt(A, B, None, 20, 0)), "ps_l1": L(1, lambda: C.gemm_pt(A, B, None, 20, 0)),
             "mainloop": lambda: C.gemm_pt(A, B, None, 35, 0)}
        t = run(v)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": f"M{M}_N{N}_K{K}", "us": t, "TF": {k: round(fl / x / 1e6) for k, x in t.items()}}), flush=True)
        del A, B
        torch.cuda.empty_cache()

    T, S, H, D, F = 257, 32, 16, 1024, 4096
    geom = AttnGeometry(T, S, 5)
    n = T + S * S - 1
    Bn = M // n
    if not only or only == "fused":
        h = torch.randn(Bn * n, D, device=dev).bfloat16()
        wq = (0.03 * torch.randn(3 * H * 64, D, device=dev)).bfloat16()
        cs = hip_ops.rope_cs_table(geom, 64, dev)
        cos, sin = hip_ops._rope_tables(geom, 64, dev)
        t = run({"hipblaslt+rope": lambda: C.rope_fwd(torch.mm(h, wq.t()).view(Bn, n, -1), cos, sin, T, S, H, False, 0.125),
                 "np_l0": L(0, lambda: C.qkv_rope_pt(h, wq, cs, T, S, H, n, False, 0.125, 0)),
                 "np_l1": L(1, lambda: C.qkv_rope_pt(h, wq, cs, T, S, H, n, False, 0.125, 0)),
                 "ps_l0": L(0, lambda: C.qkv_rope_pt(h, wq, cs, T, S, H, n, False, 0.125, 1)),
                 "ps_l1": L(1, lambda: C.qkv_rope_pt(h, wq, cs, T, S, H, n, False, 0.125, 1))})
        print(json.dumps({"op": "qkv_rope", "M": M, "us": t}), flush=True)
        del h, wq
        dy = (0.5 * torch.randn(M, D, device=dev)).bfloat16()
        w2t = (0.03 * torch.randn(F, D, device=dev)).bfloat16()
        hh = torch.randn(M, 2 * F, device=dev).bfloat16()
        def P(pf, fn):
            def f():
                C.gemm_set_prefetch(pf)
                r = fn()
                C.gemm_set_prefetch(0)
                return r
            return f

        t = run({"8ph": lambda: C.ff_dgrad_geglu(dy, w2t, hh),
                 "np_l1_pf": P(1, L(1, lambda: C.ff_dgrad_geglu_pt(dy, w2t, hh, None, 0))),
                 "ps_l1_pf": P(1, L(1, lambda: C.ff_dgrad_geglu_pt(dy, w2t, hh, None, 1))),
                 "np_l0": L(0, lambda: C.ff_dgrad_geglu_pt(dy, w2t, hh, None, 0)),
                 "np_l1": L(1, lambda: C.ff_dgrad_geglu_pt(dy, w2t, hh, None, 0)),
                 "ps_l0": L(0, lambda: C.ff_dgrad_geglu_pt(dy, w2t, hh, None, 1)),
                 "ps_l1": L(1, lambda: C.ff_dgrad_geglu_pt(dy, w2t, hh, None, 1))})
        print(json.dumps({"op": "ff_dgrad_geglu", "M": M, "us": t}), flush=True)
        del dy, w2t, hh
        torch.cuda.empty_cache()
        x = torch.randn(M, D, device=dev).bfloat16()
        w1 = (0.03 * torch.randn(2 * F, D, device=dev))
        b1 = 0.1 * torch.randn(2 * F, device=dev)
        perm = hip_ops.geglu_interleave_index(F, dev)
        w1b, b1b = w1.bfloat16(), b1.bfloat16()
        w1i, b1i = w1[perm].bfloat16().contiguous(), b1[perm].bfloat16().contiguous()
        t = run({"hipblaslt+geglu": lambda: C.geglu_fwd(torch.addmm(b1b, x, w1b.t())),
                 "np_l0": L(0, lambda: C.ff_in_geglu_pt(x, w1i, b1i, 0)),
                 "np_l1": L(1, lambda: C.ff_in_geglu_pt(x, w1i, b1i, 0)),
                 "ps": lambda: C.ff_in_geglu_pt(x, w1i, b1i, 1)})
        print(json.dumps({"op": "ff_in_geglu", "M": M, "us": t}), flush=True)
    C.gemm_set_lines(1)


if __name__ == "__main__":
    main()
