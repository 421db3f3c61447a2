#!/usr/bin/env python3
"""Split-K weight-gradient products at the bench24 micro-batch-128 shapes (M = 163840 tokens) in the
production token-contiguous forms (hip_ops._weight_grad_t): torch.bmm (hipBLASLt's heuristic pick) vs every
hipBLASLt solution for the same problem (csrc/blaslt/lt_tuned.cpp). One JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops import hip_ops  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    C = hip_ops.C()
    dev = torch.device("cuda")
    M = int(os.environ.get("M", 163840))
    torch.manual_seed(0)
    # (N_out, K_in, form): QKV / FF-in from X^T, FF-out from G^T (production forms at the bench defaults)
    for N, K, form in [(3072, 1024, "xt"), (8192, 1024, "xt"), (1024, 4096, "gt")]:
        s = hip_ops.wgrad_t_splits(M, N, K, form)
        ms = M // s
        g2 = torch.randn(M, N, device=dev).bfloat16()
        x2 = torch.randn(M, K, device=dev).bfloat16()
        if form == "xt":
            xt = x2.t().contiguous()
            a, b = g2.view(s, ms, N).transpose(1, 2), xt.view(K, s, ms).transpose(0, 1).transpose(1, 2)
        else:
            gt = g2.t().contiguous()
            a, b = gt.view(N, s, ms).transpose(0, 1), x2.view(s, ms, K)
        out = torch.empty(s, N, K, device=dev)
        t_bmm = timed(lambda: torch.bmm(a, b, out_dtype=torch.float32))
        res = C.lt_bmm_survey(a, b, out, 3)
        ok = [r for r in res if r[2]]
        best = min(ok, key=lambda r: r[1])
        fl = 2.0 * M * N * K
        print(json.dumps({"shape": f"N{N}_K{K}_M{M}", "form": form, "splits": s, "solutions": len(res), "reproducible": len(ok),
                          "torch_bmm_us": round(t_bmm, 1), "heuristic_us": round(res[0][1], 1), "best_us": round(best[1], 1),
                          "best_TF": round(fl / best[1] / 1e6), "bmm_TF": round(fl / t_bmm / 1e6), "best_index": best[0],
                          "best_kernel": best[3][:100]}), flush=True)
        del g2, x2, a, b, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
