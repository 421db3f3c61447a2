#!/usr/bin/env python3
"""The fused decode sampler (csrc/kernels/sample.hip) alone: us per call at the decode shape (32 or 64 rows x 8192
image logits), for top-k 256 / no filter / greedy, to see where its time goes."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops.hip_ops import C  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    res = {}
    for B in (32, 64):
        logits = torch.randn(B, 8192, device=dev) * 3
        seed = torch.tensor(7, dtype=torch.int64, device=dev)
        pos = torch.tensor(300, dtype=torch.int32, device=dev)
        for name, (k, p, t) in {"topk256": (256, 1.0, 1.0), "nofilter": (0, 1.0, 1.0), "greedy": (0, 1.0, 0.0),
                                "topk256_greedy": (256, 1.0, 0.0), "topk256_topp0.9": (256, 0.9, 1.0)}.items():
            for _ in range(10):
                C().sample_step(logits, k, p, t, seed, pos)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(200):
                C().sample_step(logits, k, p, t, seed, pos)
            e1.record()
            torch.cuda.synchronize()
            res[f"B{B}_{name}"] = round(e0.elapsed_time(e1) / 200 * 1e3, 2)
    print(json.dumps({"sampler_us_per_call": res}), flush=True)


if __name__ == "__main__":
    main()
