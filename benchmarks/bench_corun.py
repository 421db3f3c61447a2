#!/usr/bin/env python3
"""Can a memory-bound kernel run UNDER a compute-bound GEMM? Times (a) a GEMM alone, (b) a stream of
bandwidth-bound kernels alone, (c) both back to back on one stream and (d) both on two streams at once.
The hand-written GEMMs (gemm_pt, 8 waves x ~234 VGPRs, 130 KiB LDS per CU) leave room for one more
low-register wave per SIMD; hipBLASLt's kernels fill the register file. If (d) ~ max(a, b) the two
co-reside; if (d) ~ (c) they only time-share CUs. Device-timed, median of rounds. One JSON line per pair."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.ops import hip_ops  # noqa: E402


def timed(fn, rounds=5):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3)
    return round(statistics.median(out), 1)


def main():
    C = hip_ops.C()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M = int(os.environ.get("M", 163840))
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    A = torch.randn(M, 1024, device=dev).bfloat16()
    B = torch.randn(8192, 1024, device=dev).bfloat16()
    X = torch.randn(M, 1024, device=dev).bfloat16()  # transpose input (the LN-output -> X^T pass)
    H = torch.randn(M // 2, 8192, device=dev).bfloat16()  # geglu_fwd input (half the micro-batch)

    gemms = {"own_np": lambda: C.gemm_pt(A, B, None, 30, 0), "own_ps": lambda: C.gemm_pt(A, B, None, 20, 0),
             "hipblaslt": lambda: torch.mm(A, B.t())}
    mems = {"transpose_x8": lambda: [C.transpose_act_bf16(X) for _ in range(8)],
            "geglu_fwd_x2": lambda: [C.geglu_fwd(H) for _ in range(2)]}
    for gn, gf in gemms.items():
        for mn, mf in mems.items():
            def seq():
                gf()
                mf()

            def conc():
                cur = torch.cuda.current_stream()
                s1.wait_stream(cur)
                s2.wait_stream(cur)
                with torch.cuda.stream(s1):
                    gf()
                with torch.cuda.stream(s2):
                    mf()
                cur.wait_stream(s1)
                cur.wait_stream(s2)

            t = {"gemm": timed(gf), "mem": timed(mf), "sequential": timed(seq), "concurrent": timed(conc)}
            t["overlap_frac"] = round((t["sequential"] - t["concurrent"]) / max(1e-9, min(t["gemm"], t["mem"])), 3)
            print(json.dumps({"gemm": gn, "mem": mn, "us": t}), flush=True)


if __name__ == "__main__":
    main()
