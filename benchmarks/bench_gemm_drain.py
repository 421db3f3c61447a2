#!/usr/bin/env python3
"""End-of-workgroup store drain (gemm_set_drain: s_waitcnt vmcnt(0) after the epilogue) on every
hand-written GEMM at the bench24 B48 training shapes (M = 61440), against hipBLASLt, in interleaved
rounds in one process (median of rounds). Outputs are checked bitwise equal between drain 0 and 1."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops import hip_ops  # noqa: E402
from dalle_amd.models.patterns import AttnGeometry  # noqa: E402


def run(variants, rounds=7, reps=5):
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
    M = int(os.environ.get("M", 61440))

    def d(v, fn):
        def f():
            C.gemm_set_drain(v)
            return fn()
        return f

    for N, K in [(3072, 1024), (1024, 1024), (8192, 1024), (1024, 4096), (1024, 8192), (1024, 3072)]:
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(N, K, device=dev).bfloat16()
        for var in (300, ):
            assert torch.equal(d(0, lambda: C.gemm_nt(A, B, None, var))(), d(1, lambda: C.gemm_nt(A, B, None, var))())
        assert torch.equal(d(0, lambda: C.gemm_pt(A, B, None, 30, 0))(), d(1, lambda: C.gemm_pt(A, B, None, 30, 0))())
        v = {"hipblaslt": lambda: torch.mm(A, B.t())}
        for dr in (0, 1):
            v[f"8ph_d{dr}"] = d(dr, lambda: C.gemm_nt(A, B, None, 300))
            v[f"np_d{dr}"] = d(dr, lambda: C.gemm_pt(A, B, None, 30, 0))
            v[f"persist_d{dr}"] = d(dr, lambda: C.gemm_pt(A, B, None, 20, 0))
        v["np_mainloop"] = lambda: C.gemm_pt(A, B, None, 35, 0)
        t = run(v)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": f"M{M}_N{N}_K{K}", "us": t, "TF": {k: round(fl / x / 1e6) for k, x in t.items()}}), flush=True)
        del A, B
        torch.cuda.empty_cache()

    # weight grads dW (N, K) = G^T X over M tokens: hipBLASLt split-K bmm + fold vs the MN-major kernel
    for N, K in [(3072, 1024), (1024, 1024), (8192, 1024), (1024, 4096)]:
        G = torch.randn(M, N, device=dev).bfloat16()
        X = torch.randn(M, K, device=dev).bfloat16()
        out = torch.zeros(N, K, device=dev)
        s = hip_ops.wgrad_splits(M, N, K)
        so = max(1, min(16, 256 // ((N // 256) * (K // 256))))
        while so > 1 and M % (64 * so):
            so -= 1

        def blt():
            part = torch.bmm(G.view(s, M // s, N).transpose(1, 2), X.view(s, M // s, K), out_dtype=torch.float32)
            C.splitk_accum_(out, part, True)

        v = {"hipblaslt_splitk": blt}
        for dr in (0, 1):
            v[f"own_d{dr}"] = d(dr, lambda: C.gemm_wgrad_(G, X, out, so, True))
        t = run(v)
        fl = 2.0 * M * N * K
        print(json.dumps({"wgrad": f"M{M}_N{N}_K{K}", "splits": [s, so], "us": t,
                          "TF": {k: round(fl / x / 1e6) for k, x in t.items()}}), flush=True)
        del G, X, out
        torch.cuda.empty_cache()

    T, S, H, D, F = 257, 32, 16, 1024, 4096
    geom = AttnGeometry(T, S, 5)
    n = T + S * S - 1
    Bn = M // n
    h = torch.randn(Bn * n, D, device=dev).bfloat16()
    wq = (0.03 * torch.randn(3 * H * 64, D, device=dev)).bfloat16()
    cos, sin = hip_ops._rope_tables(geom, 64, dev)
    cs = hip_ops.rope_cs_table(geom, 64, dev)
    v = {"hipblaslt+rope": lambda: C.rope_fwd(torch.mm(h, wq.t()).view(Bn, n, -1), cos, sin, T, S, H, False, 0.125)}
    for dr in (0, 1):
        v[f"qkv_rope_8ph_d{dr}"] = d(dr, lambda: C.qkv_rope(h, wq, cos, sin, T, S, H, n, False, 0.125))
        v[f"qkv_rope_pt_d{dr}"] = d(dr, lambda: C.qkv_rope_pt(h, wq, cs, T, S, H, n, False, 0.125))
    print(json.dumps({"op": "qkv_rope", "us": run(v)}), flush=True)

    w1 = (0.03 * torch.randn(2 * F, D, device=dev))
    b1 = 0.1 * torch.randn(2 * F, device=dev)
    perm = hip_ops.geglu_interleave_index(F, dev)
    w1b, b1b = w1.bfloat16(), b1.bfloat16()
    w1i, b1i = w1[perm].bfloat16().contiguous(), b1[perm].bfloat16().contiguous()
    v = {"hipblaslt+geglu": lambda: C.geglu_fwd(torch.addmm(b1b, h, w1b.t()))}
    for dr in (0, 1):
        v[f"ff_in_geglu_pt_d{dr}"] = d(dr, lambda: C.ff_in_geglu_pt(h, w1i, b1i))
    print(json.dumps({"op": "ff_in_geglu", "us": run(v)}), flush=True)

    dy = (0.5 * torch.randn(Bn * n, D, device=dev)).bfloat16()
    w2t = (0.03 * torch.randn(F, D, device=dev)).bfloat16()
    a = torch.randn(Bn * n, 2 * F, device=dev).bfloat16()
    v = {}
    for dr in (0, 1):
        v[f"ff_dgrad_geglu_8ph_d{dr}"] = d(dr, lambda: C.ff_dgrad_geglu(dy, w2t, a, None, 0))
        v[f"ff_dgrad_geglu_pt_d{dr}"] = d(dr, lambda: C.ff_dgrad_geglu_pt(dy, w2t, a))
    print(json.dumps({"op": "ff_dgrad_geglu", "us": run(v)}), flush=True)
    C.gemm_set_drain(1)


if __name__ == "__main__":
    main()
