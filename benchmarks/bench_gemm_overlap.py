#!/usr/bin/env python3
"""Persistent register-epilogue GEMM (csrc/kernels/gemm_pt.hip) with the epilogue stores overlapped with the
next tile's first K-step (gemm_set_pt_overlap) and an optional start stagger, against hipBLASLt, the
one-tile-per-workgroup form and the main loop alone, at the bench24 micro-batch-128 token count
(M = 163840; env M). Interleaved rounds in one process, median. One JSON line per shape."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops import hip_ops  # noqa: E402


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

    def O(ovl, stag, fn):
        def f():
            C.gemm_set_pt_overlap(ovl, stag)
            r = fn()
            C.gemm_set_pt_overlap(1, 0)
            return r
        return f

    for N, K in [(3072, 1024), (8192, 1024), (4096, 1024), (1024, 1024), (1024, 4096)]:
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(N, K, device=dev).bfloat16()
        ref = torch.mm(A, B.t())
        for ovl, stag in [(0, 0), (1, 0), (1, 50), (1, 100)]:
            got = O(ovl, stag, lambda: C.gemm_pt(A, B, None, 20, 0))()
            err = ((got.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
            assert err < 1e-2, (N, K, ovl, stag, err)
        v = {"hipblaslt": lambda: torch.mm(A, B.t()), "np": lambda: C.gemm_pt(A, B, None, 30, 0),
             "ps_ovl0": O(0, 0, lambda: C.gemm_pt(A, B, None, 20, 0)),
             "ps_ovl1": O(1, 0, lambda: C.gemm_pt(A, B, None, 20, 0)),
             "ps_ovl1_stag50": O(1, 50, lambda: C.gemm_pt(A, B, None, 20, 0)),
             "ps_ovl1_stag100": O(1, 100, lambda: C.gemm_pt(A, B, None, 20, 0)),
             "ps_ovl0_stag100": O(0, 100, lambda: C.gemm_pt(A, B, None, 20, 0)),
             "mainloop": lambda: C.gemm_pt(A, B, None, 25, 0)}
        t = run(v)
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": f"M{M}_N{N}_K{K}", "us": t, "TF": {k: round(fl / x / 1e6) for k, x in t.items()}}), flush=True)
        del A, B, ref
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
