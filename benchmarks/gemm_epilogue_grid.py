#!/usr/bin/env python3
"""Persistent GEMM epilogue cost vs the number of concurrently storing CUs: the same kernel with its
grid capped at 32 / 64 / 128 / 256 workgroups (DALLE_AMD_PT_GRID, read per launch), full epilogue (gemm_pt
variant 20) vs main loop only (25). Per-tile epilogue cost = (full - mainloop) / tiles per workgroup.
If it falls with fewer storers the cost is the chip's aggregate write path; if not, a per-CU limit."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops import hip_ops  # noqa: E402


def timed(fn, rounds=5, reps=3):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3 / reps)
    return statistics.median(out)


def main():
    C = hip_ops.C()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M = 61440
    for N, K in [(3072, 1024), (1024, 4096)]:
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(N, K, device=dev).bfloat16()
        tiles = (M // 256) * (N // 256)
        res = {"shape": f"M{M}_N{N}_K{K}"}
        for grid in (32, 64, 128, 256):
            os.environ["DALLE_AMD_PT_GRID"] = str(grid)
            full = timed(lambda: C.gemm_pt(A, B, None, 20, 0))
            main_ = timed(lambda: C.gemm_pt(A, B, None, 25, 0))
            per = tiles / grid
            res[f"g{grid}"] = {"full_us": round(full, 1), "mainloop_us": round(main_, 1),
                               "epi_us_per_tile": round((full - main_) / per, 2), "tiles_per_wg": round(per, 2)}
        os.environ.pop("DALLE_AMD_PT_GRID")
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
