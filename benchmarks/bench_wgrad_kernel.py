#!/usr/bin/env python3
"""Repeated launches of one weight-grad shape for counter collection (rocprofv3 --pmc): the
hand-written MN-major kernel (gemm_wgrad_) and hipBLASLt's split-K batched GEMM side by side, plus the
NT kernel on the transposed problem for reference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops.ext import load_extension  # noqa: E402


def main():
    C = load_extension(required=True)
    M, N, K, s = (int(v) for v in (sys.argv[1:5] if len(sys.argv) > 4 else (61440, 1024, 4096, 4)))
    dev = torch.device("cuda")
    g = torch.randn(M, N, device=dev).bfloat16()
    x = torch.randn(M, K, device=dev).bfloat16()
    acc = torch.zeros(N, K, device=dev)
    gt, xt = g.t().contiguous(), x.t().contiguous()
    for _ in range(10):
        C.gemm_wgrad_(g, x, acc, s, True)
        part = torch.bmm(g.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K), out_dtype=torch.float32)
        C.splitk_accum_(acc, part, True)
        C.gemm_nt(gt, xt, None, 300)
    torch.cuda.synchronize()
    print("done", M, N, K, s)


if __name__ == "__main__":
    main()
