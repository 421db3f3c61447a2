#!/usr/bin/env python3
"""Cache policy of the hand-written GEMMs' output stores (common.h cstore16) at the bench24 B48 training
shapes (M = 61440 tokens), random operands, interleaved rounds in one process (median of rounds).

cpol: 0 plain flat store, 2 nt, 16 sc1, 17 sc0 sc1 (sc1 forms drop the written line from the XCD L2, so
the output tiles do not evict the operand panels the next tiles stream from). Every policy must produce
bitwise the same output; the script checks that before timing.
"""
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


def with_cpol(C, cp, fn):
    def f():
        C.gemm_set_cpol(cp)
        return fn()
    return f


def main():
    C = hip_ops.C()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M = int(os.environ.get("M", 61440))
    pols = [int(p) for p in os.environ.get("CPOLS", "0,2,16,17").split(",")]
    shapes = [(3072, 1024), (1024, 1024), (8192, 1024), (4096, 1024), (1024, 4096), (1024, 8192)]
    for N, K in shapes:
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(N, K, device=dev).bfloat16()
        ref8 = with_cpol(C, 0, lambda: C.gemm_nt(A, B, None, 300))()
        refp = with_cpol(C, 0, lambda: C.gemm_pt(A, B, None, 30, 0))()
        for cp in pols:
            assert torch.equal(with_cpol(C, cp, lambda: C.gemm_nt(A, B, None, 300))(), ref8), f"8ph cpol {cp}"
            assert torch.equal(with_cpol(C, cp, lambda: C.gemm_pt(A, B, None, 30, 0))(), refp), f"pt cpol {cp}"
            assert torch.equal(with_cpol(C, cp, lambda: C.gemm_pt(A, B, None, 20, 0))(), refp), f"pt persist cpol {cp}"
        del ref8, refp
        v = {"hipblaslt": lambda: torch.mm(A, B.t())}
        for cp in pols:
            v[f"8ph_c{cp}"] = with_cpol(C, cp, lambda: C.gemm_nt(A, B, None, 300))
            v[f"np_c{cp}"] = with_cpol(C, cp, lambda: C.gemm_pt(A, B, None, 30, 0))
            v[f"persist_c{cp}"] = with_cpol(C, cp, lambda: C.gemm_pt(A, B, None, 20, 0))
        v["np_mainloop"] = lambda: C.gemm_pt(A, B, None, 35, 0)
        t = run(v)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": f"M{M}_N{N}_K{K}", "us": t, "TF": {k: round(fl / x / 1e6) for k, x in t.items()}}), flush=True)
        del A, B
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
    for cp in pols:
        v[f"qkv_rope_8ph_c{cp}"] = with_cpol(C, cp, lambda: C.qkv_rope(h, wq, cos, sin, T, S, H, n, False, 0.125))
        v[f"qkv_rope_pt_c{cp}"] = with_cpol(C, cp, lambda: C.qkv_rope_pt(h, wq, cs, T, S, H, n, False, 0.125))
    print(json.dumps({"op": "qkv_rope", "us": run(v)}), flush=True)

    w1 = (0.03 * torch.randn(2 * F, D, device=dev))
    b1 = 0.1 * torch.randn(2 * F, device=dev)
    perm = hip_ops.geglu_interleave_index(F, dev)
    w1b, b1b = w1.bfloat16(), b1.bfloat16()
    w1i, b1i = w1[perm].bfloat16().contiguous(), b1[perm].bfloat16().contiguous()
    v = {"hipblaslt+geglu": lambda: C.geglu_fwd(torch.addmm(b1b, h, w1b.t()))}
    for cp in pols:
        v[f"ff_in_geglu_pt_c{cp}"] = with_cpol(C, cp, lambda: C.ff_in_geglu_pt(h, w1i, b1i))
        v[f"ff_in_geglu_persist_c{cp}"] = with_cpol(C, cp, lambda: C.ff_in_geglu_pt(h, w1i, b1i, 1))
    print(json.dumps({"op": "ff_in_geglu", "us": run(v)}), flush=True)

    dy = (0.5 * torch.randn(Bn * n, D, device=dev)).bfloat16()
    w2t = (0.03 * torch.randn(F, D, device=dev)).bfloat16()
    a = torch.randn(Bn * n, 2 * F, device=dev).bfloat16()
    v = {}
    for cp in pols:
        v[f"ff_dgrad_geglu_8ph_c{cp}"] = with_cpol(C, cp, lambda: C.ff_dgrad_geglu(dy, w2t, a, None, 0))
        v[f"ff_dgrad_geglu_pt_c{cp}"] = with_cpol(C, cp, lambda: C.ff_dgrad_geglu_pt(dy, w2t, a))
    print(json.dumps({"op": "ff_dgrad_geglu", "us": run(v)}), flush=True)
    C.gemm_set_cpol(0)


if __name__ == "__main__":
    main()
