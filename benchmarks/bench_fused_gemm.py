#!/usr/bin/env python3
"""Median time of the two fused-epilogue GEMMs at the bench24 B48 shapes (M = 61440 tokens):
FF-out dgrad + GEGLU backward (ff_dgrad_geglu) and QKV + rotary into the attention layout (qkv_rope).
One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.models.rotary import rotary_tables  # noqa: E402
from dalle_amd.ops.ext import load_extension  # noqa: E402


def timeit(fn, reps=20, warmup=3):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2] * 1e3


def main():
    C = load_extension(required=True)
    dev = torch.device("cuda")
    M, D, F, H, T, S = 61440, 1024, 4096, 16, 257, 32
    n = T + S * S - 1
    dy = torch.randn(M, D, device=dev).bfloat16()
    w2t = (torch.randn(F, D, device=dev) * 0.03).bfloat16()
    h = torch.randn(M, 2 * F, device=dev).bfloat16()
    x = torch.randn(M, D, device=dev).bfloat16()
    wq = (torch.randn(3 * H * 64, D, device=dev) * 0.03).bfloat16()
    cos, sin = rotary_tables(T, S, 64, device=dev)
    res = {}
    res["ff_dgrad_geglu_us"] = round(timeit(lambda: C.ff_dgrad_geglu(dy, w2t, h)), 1)
    res["qkv_rope_us"] = round(timeit(lambda: C.qkv_rope(x, wq, cos, sin, T, S, H, n, False, 0.125)), 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
