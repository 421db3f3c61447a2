#!/usr/bin/env python3
"""Where the hand-written 8-phase GEMM's time goes at the training shapes (M = 61440): the full kernel
(variant 300), the same main loop with no epilogue (350: accumulators kept live, nothing stored) and with
the LDS staging of the epilogue but no global stores (360), against hipBLASLt's NT form."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.bench_gemm_layouts import timeit  # noqa: E402
from dalle_amd.ops.ext import load_extension  # noqa: E402


def main():
    C = load_extension(required=True)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M = int(os.environ.get("M", 61440))
    for N, K in [(3072, 1024), (1024, 1024), (8192, 1024), (4096, 1024), (1024, 4096)]:
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(N, K, device=dev).bfloat16()
        fl = 2.0 * M * N * K
        res = {"shape": f"M{M}_N{N}_K{K}", "hipblaslt_NT_us": round(timeit(lambda: torch.mm(A, B.t())) * 1e3, 1)}
        for v, name in ((300, "full_us"), (370, "full_nt_store_us"), (360, "no_global_store_us"), (350, "no_epilogue_us")):
            res[name] = round(timeit(lambda: C.gemm_nt(A, B, None, v)) * 1e3, 1)
        res["full_TF"] = round(fl / res["full_us"] / 1e6)
        res["no_epilogue_TF"] = round(fl / res["no_epilogue_us"] / 1e6)
        res["hipblaslt_TF"] = round(fl / res["hipblaslt_NT_us"] / 1e6)
        print(json.dumps(res), flush=True)
        del A, B
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
