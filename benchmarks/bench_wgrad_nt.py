"""Weight-gradient GEMMs at micro-batch 64 (M = 81920 tokens): the production split-K form over token-major
operands (g^T x, both operands contiguous along the output dims: the MFMA loads need a transpose) against
the same product over pre-transposed, token-contiguous operands (G^T [N, M], X^T [K, M]: the "NT" form the
forward / input-grad GEMMs run in), at every split factor. Prices what producers that also emit transposed
activations would buy; the standalone transpose is timed too (what a non-fused producer would pay).
Prints one JSON line per shape (TF/s = 2 M N K / time)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops.ext import load_extension  # noqa: E402
from dalle_amd.ops.hip_ops import wgrad_splits  # noqa: E402

C = load_extension(required=True)


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
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


M = int(os.environ.get("WGRAD_M", "81920"))
dev = "cuda"
for N, K in [(3072, 1024), (1024, 1024), (8192, 1024), (1024, 4096)]:
    g = torch.randn(M, N, device=dev).bfloat16()
    x = torch.randn(M, K, device=dev).bfloat16()
    fl = 2 * M * N * K
    s0 = wgrad_splits(M, N, K)
    r = {"shape": f"M{M}_N{N}_K{K}", "prod_splits": s0}
    r["prod_TF"] = round(fl / timeit(lambda: torch.bmm(g.view(s0, M // s0, N).transpose(1, 2), x.view(s0, M // s0, K),
                                                       out_dtype=torch.float32)) / 1e9)
    gt = g.t().contiguous()  # [N, M]
    xt = x.t().contiguous()  # [K, M]
    r["transpose_us"] = {"g": round(timeit(lambda: g.t().contiguous()) * 1e3, 1),
                         "x": round(timeit(lambda: x.t().contiguous()) * 1e3, 1),
                         "x_hip": round(timeit(lambda: C.transpose_act_bf16(x)) * 1e3, 1)}
    best = None
    for s in (1, 2, 4, 8, 16):
        ms = M // s
        a = gt.view(N, s, ms).transpose(0, 1)                  # [s, N, ms], token-contiguous rows
        bt = xt.view(K, s, ms).transpose(0, 1).transpose(1, 2)  # [s, ms, K], token-contiguous columns
        tf = round(fl / timeit(lambda: torch.bmm(a, bt, out_dtype=torch.float32)) / 1e9)
        r[f"nt_s{s}_TF"] = tf
        best = max(best or 0, tf)
    r["nt_best_TF"] = best
    # one operand transposed: token-contiguous G^T with token-major x, and token-major g with X^T
    for name in ("gT_only", "xT_only"):
        bestm = 0
        for s in (2, 4, 8, 16):
            ms = M // s
            if name == "gT_only":
                a = gt.view(N, s, ms).transpose(0, 1)
                b = x.view(s, ms, K)
            else:
                a = g.view(s, ms, N).transpose(1, 2)
                b = xt.view(K, s, ms).transpose(0, 1).transpose(1, 2)
            tf = round(fl / timeit(lambda: torch.bmm(a, b, out_dtype=torch.float32)) / 1e9)
            r[f"{name}_s{s}_TF"] = tf
            bestm = max(bestm, tf)
        r[f"{name}_best_TF"] = bestm
    print(json.dumps(r), flush=True)
    del g, x, gt, xt
    torch.cuda.empty_cache()
