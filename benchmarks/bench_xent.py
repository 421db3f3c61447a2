#!/usr/bin/env python3
"""Fused cross-entropy + bias-gradient kernel (xent_colsum_) per head chunk at the bench24 micro-batch-64
shapes: the text chunk (16384 x 32356) and an image chunk (16384 x 8192), against a same-bytes
read+write pass (the HBM roofline of an in-place softmax-gradient) and the column-sum fold alone.
Interleaved rounds, median (us)."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops import hip_ops  # noqa: E402


def run(variants, rounds=7, reps=5):
    res = {k: [] for k in variants}
    for fn in variants.values():
        fn()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, fn in variants.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                fn()
            b.record()
            torch.cuda.synchronize()
            res[k].append(a.elapsed_time(b) * 1e3 / reps)
    return {k: round(statistics.median(v), 1) for k, v in res.items()}


def main():
    C = hip_ops.C()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    R = int(os.environ.get("ROWS", 16384))
    for V in (32356, 8192):
        base = (2.0 * torch.randn(R, V, device=dev)).bfloat16()
        logit = base.clone()
        lab = torch.randint(0, V, (R,), device=dev)
        db = torch.zeros(V, device=dev)
        dst = torch.empty_like(base)
        nbytes = 2 * base.numel() * 2

        def fused():
            return C.xent_colsum_(logit, lab, 1.0 / R, db)

        def nocol():
            return C.xent_fwd_bwd_(logit, lab, 1.0 / R)

        def copy():
            dst.copy_(base)

        t = run({"xent_colsum": fused, "xent_fwd_bwd_no_colsum": nocol, "copy_same_bytes": copy})
        res = {"shape": f"{R}x{V}", "us": t, "GBps": {k: round(nbytes / v / 1e3) for k, v in t.items()}}
        print(json.dumps(res), flush=True)
        del base, logit, dst
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
