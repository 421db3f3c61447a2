#!/usr/bin/env python3
"""Persistent GEMM family (csrc/kernels/gemm_pt.hip) vs hipBLASLt and the one-tile-per-workgroup 8-phase
kernel at the bench24 B48 training shapes (M = 61440 tokens), random operands. Variants are timed in
interleaved rounds in one process (median of rounds); one JSON line per shape / fused op.

  plain:  hipBLASLt NT | 8-phase (gemm_nt 300) | persistent (gemm_pt) | persistent main loop only (variant 5)
  fused:  QKV + rotary, FF-in + GEGLU, FF-out dgrad + GEGLU backward against their current paths
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


def main():
    C = hip_ops.C()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M = int(os.environ.get("M", 61440))
    groups = [int(g) for g in os.environ.get("PT_GROUPS", "0").split(",")]
    shapes = [(3072, 1024), (1024, 1024), (8192, 1024), (4096, 1024), (1024, 4096), (1024, 8192), (1024, 3072)]
    if os.environ.get("PT_FUSED_ONLY"):
        shapes = []
    for N, K in shapes:
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(N, K, device=dev).bfloat16()
        v = {"hipblaslt": lambda: torch.mm(A, B.t()), "8ph": lambda: C.gemm_nt(A, B, None, 300),
             "8ph_stagger": lambda: C.gemm_nt(A, B, None, 390)}
        for g in groups:
            v[f"np_stagger_g{g}"] = (lambda g=g: C.gemm_pt(A, B, None, 10, g))
            v[f"np_g{g}"] = (lambda g=g: C.gemm_pt(A, B, None, 30, g))
        v["np_mainloop"] = lambda: C.gemm_pt(A, B, None, 35, 0)
        t = run(v)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": f"M{M}_N{N}_K{K}", "us": t, "TF": {k: round(fl / x / 1e6) for k, x in t.items()}}), flush=True)
        del A, B
        torch.cuda.empty_cache()

    # fused ops at the bench24 geometry (T = 257, 32 x 32 image, 16 heads)
    T, S, H, D, F = 257, 32, 16, 1024, 4096
    geom = AttnGeometry(T, S, 5)
    n = T + S * S - 1
    B = M // n
    h = torch.randn(B * n, D, device=dev).bfloat16()
    wq = (0.03 * torch.randn(3 * H * 64, D, device=dev)).bfloat16()
    cos, sin = hip_ops._rope_tables(geom, 64, dev)
    cs = hip_ops.rope_cs_table(geom, 64, dev)
    t = run({"qkv_rope_8ph": lambda: C.qkv_rope(h, wq, cos, sin, T, S, H, n, False, 0.125),
             "qkv_rope_pt": lambda: C.qkv_rope_pt(h, wq, cs, T, S, H, n, False, 0.125),
             "qkv_rope_pt_persist": lambda: C.qkv_rope_pt(h, wq, cs, T, S, H, n, False, 0.125, 1),
             "hipblaslt+rope": lambda: C.rope_fwd(torch.mm(h, wq.t()).view(B, n, -1), cos, sin, T, S, H, False, 0.125)})
    print(json.dumps({"op": "qkv_rope", "us": t}), flush=True)

    w1 = (0.03 * torch.randn(2 * F, D, device=dev))
    b1 = 0.1 * torch.randn(2 * F, device=dev)
    perm = hip_ops.geglu_interleave_index(F, dev)
    w1b, b1b = w1.bfloat16(), b1.bfloat16()
    w1i, b1i = w1[perm].bfloat16().contiguous(), b1[perm].bfloat16().contiguous()
    t = run({"hipblaslt+geglu": lambda: C.geglu_fwd(torch.addmm(b1b, h, w1b.t())),
             "ff_in_geglu_pt": lambda: C.ff_in_geglu_pt(h, w1i, b1i),
             "ff_in_geglu_pt_persist": lambda: C.ff_in_geglu_pt(h, w1i, b1i, 1)})
    print(json.dumps({"op": "ff_in_geglu", "us": t}), flush=True)

    dy = (0.5 * torch.randn(B * n, D, device=dev)).bfloat16()
    w2t = (0.03 * torch.randn(F, D, device=dev)).bfloat16()
    a = torch.randn(B * n, 2 * F, device=dev).bfloat16()
    t = run({"ff_dgrad_geglu_8ph": lambda: C.ff_dgrad_geglu(dy, w2t, a, None, 0),
             "ff_dgrad_geglu_8ph_stagger": lambda: C.ff_dgrad_geglu(dy, w2t, a, None, -1),
             "ff_dgrad_geglu_pt": lambda: C.ff_dgrad_geglu_pt(dy, w2t, a),
             "ff_dgrad_geglu_pt_persist": lambda: C.ff_dgrad_geglu_pt(dy, w2t, a, None, 1)})
    print(json.dumps({"op": "ff_dgrad_geglu", "us": t}), flush=True)


if __name__ == "__main__":
    main()
