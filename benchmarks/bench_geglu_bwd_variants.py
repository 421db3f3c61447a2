#!/usr/bin/env python3
"""FF-out dgrad + GEGLU backward at the bench24 micro-batch-128 shape (M = 163840, F = 4096, K = 1024):
the 8-phase kernel (LDS-staged epilogue, the default through round 4), the register-epilogue kernel one
tile per workgroup (its GEGLU epilogue through LDS, pt_epilogue_geglu_bwd_lds) and persistent, and the
plain products (hipBLASLt, register-epilogue main loop only). Device-timed, interleaved rounds, median."""
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
    t = run({"8ph": lambda: C.ff_dgrad_geglu(dy, w2t, h), "pt_tile_lds": lambda: C.ff_dgrad_geglu_pt(dy, w2t, h, None, 0),
             "pt_persist": lambda: C.ff_dgrad_geglu_pt(dy, w2t, h, None, 1),
             "plain_hipblaslt": lambda: torch.mm(dy, w2t.t()), "pt_mainloop": lambda: C.gemm_pt(dy, w2t, None, 35, 0)})
    print(json.dumps({"M": M, "F": F, "K": K, "us": t}), flush=True)
    del dy, w2t, h
    # FF-in + GEGLU forward: hipBLASLt addmm + the GEGLU pass (default) vs the register-epilogue kernel one
    # tile per workgroup (GEGLU through LDS) and persistent
    x = torch.randn(M, K, device=dev).bfloat16()
    w1i = (0.03 * torch.randn(2 * F, K, device=dev)).bfloat16()
    b1i = (0.1 * torch.randn(2 * F, device=dev)).bfloat16()
    t = run({"hipblaslt_geglu": lambda: C.geglu_fwd(torch.addmm(b1i, x, w1i.t())),
             "pt_tile_lds": lambda: C.ff_in_geglu_pt(x, w1i, b1i, 0), "pt_persist": lambda: C.ff_in_geglu_pt(x, w1i, b1i, 1)})
    print(json.dumps({"op": "ff_in_geglu", "M": M, "F": F, "K": K, "us": t}), flush=True)


if __name__ == "__main__":
    main()
