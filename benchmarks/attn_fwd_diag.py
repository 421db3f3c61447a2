#!/usr/bin/env python3
"""Standalone timing of the training attention forward (bench24 micro-batch: B=48, T=257, 32x32 image,
16 heads) for the three layer patterns. With DALLE_AMD_ATTN_DIAG set the kernel SKIPS parts of its work
(measurement only, wrong outputs): 1 = phase A's text-tile staging, 2 = phase A's barriers, 4 = phase B's
local tiles; the time difference is what each part costs.

    DALLE_AMD_ATTN_DIAG=4 python benchmarks/attn_fwd_diag.py
"""
import json
import os
import sys

import torch
sys.path.insert(0, os.getcwd())
from dalle_amd.ops.ext import load_extension
C = load_extension(required=True)
dev = torch.device("cuda")
B, T, S, H = 48, 257, 32, 16
n = T + S * S - 1
Np = (T + 31) // 32 * 32 + S * S
q = torch.randn(B * H, Np, 64, device=dev).bfloat16() * 0.3
k = torch.randn_like(q); v = torch.randn_like(q)
def t(pattern):
    for _ in range(3): C.attn_fwd(q, k, v, B, T, S, n, 5, H, pattern)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20): C.attn_fwd(q, k, v, B, T, S, n, 5, H, pattern)
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / 20 * 1e3
print(json.dumps({"diag": os.environ.get("DALLE_AMD_ATTN_DIAG", "0"), "axial_row_us": round(t(1), 1), "axial_col_us": round(t(2), 1), "conv_us": round(t(3), 1)}))
