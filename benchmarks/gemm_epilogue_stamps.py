#!/usr/bin/env python3
"""Where a one-tile-per-workgroup GEMM's epilogue time goes: per-workgroup real-time stamps (10 ns
ticks) from gemm_pt variant 40 {start, epilogue start, stores issued, stores complete, CU id}, and the
kernel time with every workgroup storing (30), only even workgroups storing (41) and none (35).

If the epilogue cost is the chip's write bandwidth under synchronized bursts, halving the storing
workgroups halves it; if it is a per-CU store cost, it does not change.
"""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops import hip_ops  # noqa: E402


def timed(fn, rounds=7, reps=5):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3 / reps)
    return round(statistics.median(out), 1)


def med(x):
    return round(float(statistics.median(x)), 2)


def main():
    C = hip_ops.C()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M = int(os.environ.get("M", 61440))
    for N, K in [(3072, 1024), (8192, 1024), (1024, 4096)]:
        A = torch.randn(M, K, device=dev).bfloat16()
        B = torch.randn(N, K, device=dev).bfloat16()
        tiles = (M // 256) * (N // 256)
        st = torch.zeros(tiles * 5, dtype=torch.long, device=dev)
        t = {"all_store": timed(lambda: C.gemm_pt(A, B, None, 30, 0)),
             "even_store": timed(lambda: C.gemm_pt(A, B, st, 41, 0)),
             "stamped": timed(lambda: C.gemm_pt(A, B, st, 40, 0)),
             "no_store": timed(lambda: C.gemm_pt(A, B, None, 35, 0))}
        res = {"shape": f"M{M}_N{N}_K{K}", "us": t}
        for var in (40, 41):
            C.gemm_pt(A, B, st, var, 0)
            torch.cuda.synchronize()
            s = st.view(tiles, 5).cpu().double()
            t0 = s[:, 0].min()
            s[:, :4] = (s[:, :4] - t0) * 0.01  # us
            main_us = (s[:, 1] - s[:, 0]).tolist()
            issue_us = (s[:, 2] - s[:, 1]).tolist()
            drain_us = (s[:, 3] - s[:, 2]).tolist()
            # how many workgroups are inside their epilogue (start .. stores complete) when one starts
            starts, ends = s[:, 1], s[:, 3]
            conc = [int(((starts <= x) & (ends > x)).sum()) for x in starts[:: max(1, tiles // 512)].tolist()]
            # spread of the first wave's epilogue starts (us)
            first = s[:256, 1]
            key = "stamps_all" if var == 40 else "stamps_even"
            res[key] = {"span_us": round(float(s[:, 3].max()), 1), "main_med": med(main_us), "issue_med": med(issue_us),
                        "drain_med": med(drain_us), "drain_p90": round(float(torch.tensor(drain_us).quantile(0.9)), 2),
                        "concurrent_epilogues_med": med(conc),
                        "first_wave_epi_start_spread_us": round(float(first.max() - first.min()), 2),
                        "cus_seen": int(s[:, 4].unique().numel())}
        print(json.dumps(res), flush=True)
        del A, B
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
