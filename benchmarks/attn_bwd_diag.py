#!/usr/bin/env python3
"""The training attention backward (rotary-fused, bench24 micro-batch B=48, T=257, 32x32 image, 16 heads) for
the three layer patterns, for a per-kernel profile (rocprofv3 --kernel-trace --stats). With DALLE_AMD_ATTN_DIAG
the kernels SKIP parts of their work (measurement only, wrong outputs): dQ 1/2/4 = text staging / barriers /
local tiles, text dK/dV 8/16 = staging / barriers.

    rocprofv3 --kernel-trace --stats -d out -- python3 benchmarks/attn_bwd_diag.py
"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from dalle_amd.ops.ext import load_extension  # noqa: E402

C = load_extension(required=True)
dev = torch.device("cuda")
B, T, S, H = 48, 257, 32, 16
n = T + S * S - 1
Np = (T + 31) // 32 * 32 + S * S
q = torch.randn(B * H, Np, 64, device=dev).bfloat16() * 0.3
k = torch.randn_like(q)
v = torch.randn_like(q)
cos = torch.randn(n, 64, device=dev)
sin = torch.randn(n, 64, device=dev)
for pattern in (1, 2, 3):
    out, lse = C.attn_fwd(q, k, v, B, T, S, n, 5, H, pattern)
    dout = torch.randn_like(out)
    for _ in range(10):
        C.attn_bwd_rope(q, k, v, out, dout, lse, cos, sin, B, T, S, n, 5, H, pattern, 1.0)
    torch.cuda.synchronize()
print("done", os.environ.get("DALLE_AMD_ATTN_DIAG", "0"))
