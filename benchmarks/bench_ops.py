#!/usr/bin/env python3
"""Per-op microbenchmarks at the bench24 shapes (B x 1280 tokens, d=1024, 16 heads): sparse attention
fwd/bwd per pattern, GEMM weight-gradient variants, and the fused elementwise kernels. Prints a
JSON line per op with the median time over interleaved repetitions (cuda events)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dalle_amd.models.patterns import AttnGeometry  # noqa: E402
from dalle_amd.ops import hip_ops  # noqa: E402


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
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--only", default="")
    ap.add_argument("--tunable", action="store_true", help="enable PyTorch TunableOp GEMM search")
    args = ap.parse_args()
    dev = torch.device("cuda")
    if args.tunable:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_filename(os.path.join("gpurun_out", "tunableop_results.csv"))
    B, H, T, S = args.batch, 16, 257, 32
    n = T + S * S - 1
    geom = AttnGeometry(T, S, 5)
    res = []
    if args.only in ("", "attn"):
        for t in ["axial_row", "axial_col", "conv_like"]:
            qkv = (torch.randn(B, n, 3 * H * 64, device=dev)).to(torch.bfloat16).requires_grad_(True)
            out = hip_ops.attention_core(qkv, H, geom, t)
            g = torch.randn_like(out)
            f_ms = timeit(lambda: hip_ops.attention_core(qkv, H, geom, t))
            b_ms = timeit(lambda: torch.autograd.grad(hip_ops.attention_core(qkv, H, geom, t), qkv, g))
            # useful FLOPs: image queries x (text + local keys) + causal text, QK^T and PV (x2 bwd)
            loc = {"axial_row": 16.5, "axial_col": 16.5, "conv_like": 13}[t]
            flops = 4 * B * H * 64 * (T * T / 2 + S * S * (T + loc))
            res.append({"op": f"attn_{t}", "fwd_ms": round(f_ms, 3), "fwd+bwd_ms": round(b_ms, 3),
                        "fwd_TFLOPs": round(flops / f_ms / 1e9, 1), "bwd_TFLOPs": round(2.5 * flops / (b_ms - f_ms) / 1e9, 1)})
    if args.only in ("", "gemm"):
        M = B * n
        for (N, K) in [(3072, 1024), (1024, 1024), (8192, 1024), (1024, 4096)]:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            g = torch.randn(M, N, device=dev).to(torch.bfloat16)
            w = torch.randn(N, K, device=dev).to(torch.bfloat16)
            acc = torch.zeros(N, K, device=dev)
            fl = 2 * M * N * K
            t_fwd = timeit(lambda: torch.mm(x, w.t()))
            t_dx = timeit(lambda: torch.mm(g, w))
            t_dw32 = timeit(lambda: torch.mm(g.t(), x, out_dtype=torch.float32))
            t_dwacc = timeit(lambda: torch.addmm(acc, g.t(), x, out_dtype=torch.float32, out=acc))
            t_dw16 = timeit(lambda: torch.mm(g.t(), x))
            t_dwT = timeit(lambda: torch.mm(x.t(), g, out_dtype=torch.float32))
            r = {"op": f"gemm_M{M}_N{N}_K{K}", "fwd_TF": round(fl / t_fwd / 1e9), "dx_TF": round(fl / t_dx / 1e9),
                 "dw_fp32out_TF": round(fl / t_dw32 / 1e9), "dw_accum_TF": round(fl / t_dwacc / 1e9),
                 "dw_bf16out_TF": round(fl / t_dw16 / 1e9), "dwT_fp32out_TF": round(fl / t_dwT / 1e9)}
            for s in (4, 8, 16):
                gs, xs = g.view(s, M // s, N).transpose(1, 2), x.view(s, M // s, K)
                try:
                    t_sk = timeit(lambda: torch.sum(torch.bmm(gs, xs, out_dtype=torch.float32), 0, out=acc))
                    r[f"dw_splitk{s}_bmm32_TF"] = round(fl / t_sk / 1e9)
                except Exception as e:  # out_dtype for bmm may be unsupported on this build
                    r[f"dw_splitk{s}_bmm32_TF"] = str(e)[:60]
                t_sk16 = timeit(lambda: torch.sum(torch.bmm(gs, xs), 0, dtype=torch.float32, out=acc))
                r[f"dw_splitk{s}_bmm16_TF"] = round(fl / t_sk16 / 1e9)
            res.append(r)
            print(json.dumps(r), flush=True)
    for r in res:
        if not r["op"].startswith("gemm"):
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
