#!/usr/bin/env python3
"""FF-out dgrad + GEGLU backward at the bench24 micro-batch-128 shape (M = 163840, F = 4096, K = 1024):
the one-workgroup-per-CU 8-phase kernel vs the two-workgroups-per-CU kernel (gemm_set_geglu_bwd_2wg), and
the plain product on both structures. Device-timed, interleaved rounds, median. One JSON line."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops import hip_ops  # noqa: E402


def run(variants, rounds=7):
    for fn in variants.values():
        fn()
    torch.cuda.synchronize()
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for k, fn in variants.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            torch.cuda.synchronize()
            res[k].append(a.elapsed_time(b) * 1e3)
    return {k: round(statistics.median(v), 1) for k, v in res.items()}


def main():
    C = hip_ops.C()
    dev = torch.device("cuda")
    M = int(os.environ.get("M", 163840))
    F, K = 4096, 1024
    torch.manual_seed(0)
    dy = (0.5 * torch.randn(M, K, device=dev)).bfloat16()
    w2t = (0.03 * torch.randn(F, K, device=dev)).bfloat16()
    h = torch.randn(M, 2 * F, device=dev).bfloat16()

    def G(v):
        def f():
            C.gemm_set_geglu_bwd_2wg(v)
            r = C.ff_dgrad_geglu(dy, w2t, h)
            C.gemm_set_geglu_bwd_2wg(0)
            return r
        return f

    t = run({"8ph": G(0), "2wg": G(1), "plain_hipblaslt": lambda: torch.mm(dy, w2t.t()), "plain_2wg": lambda: C.gemm_2wg(dy, w2t),
             "plain_8ph": lambda: C.gemm_nt(dy, w2t, None, 300)})
    print(json.dumps({"M": M, "F": F, "K": K, "us": t}), flush=True)
    # start stagger of the co-resident workgroups (10 ns ticks; fw < 0: second slot delayed, > 0: 4-phase)
    for ticks, fw in [(1500, -256), (2800, -256), (4000, -256), (1400, 512), (700, 512), (2800, -128)]:
        C.gemm_set_2wg_stagger(ticks, fw)
        t = run({"2wg": G(1), "plain_2wg": lambda: C.gemm_2wg(dy, w2t)}, rounds=5)
        print(json.dumps({"stagger": ticks, "first_wave": fw, "us": t}), flush=True)
    C.gemm_set_2wg_stagger(0, -256)


if __name__ == "__main__":
    main()
