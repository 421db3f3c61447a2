"""Leading-dimension padding A/B for the assembly GEMMs: does a power-of-two row stride (K = 1024 / 3072 /
4096 / 8192 bf16 rows are 2-16 KB apart) cost the LDS-DMA loads L2-channel or DRAM-page conflicts?

    python benchmarks/bench_ld_pad.py [--rounds 4]

Times asm_gemm (NT) and asm_wgrad_ (TN) through the built extension on operands whose rows are `pad`
elements longer than the logical width (a view of a wider buffer), interleaved in one process.
Prints one JSON line per shape: microseconds per pad."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from dalle_amd.ops.hip_ops import C, asm_wgrad_splits


def timed(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


def padded(src, pad):
    buf = torch.zeros(src.shape[0], src.shape[1] + pad, device="cuda", dtype=torch.bfloat16)
    buf[:, :src.shape[1]] = src
    return buf[:, :src.shape[1]]


def rnd(rows, cols):
    return torch.randn(rows, cols, device="cuda", dtype=torch.bfloat16) * 0.02


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--pads", default="0,64,128")
    a = ap.parse_args()
    pads = [int(p) for p in a.pads.split(",")]
    M = 163840
    for N, K in ((1024, 8192), (1024, 3072), (1024, 4096), (8192, 1024)):
        A0, B0 = rnd(M, K), rnd(N, K)
        ops = {p: (padded(A0, p), padded(B0, p)) for p in pads}
        del A0, B0
        ref = None
        res = {p: [] for p in pads}
        for _ in range(a.rounds):
            for p in pads:
                A, B = ops[p]
                out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                res[p].append(timed(lambda: C().asm_gemm(A, B, None, out)))
                if ref is None:
                    ref = out.float()
                else:
                    assert torch.equal(out.float(), ref), "padded operands changed the result"
        ref = None
        print(json.dumps({"kind": "nt", "M": M, "N": N, "K": K,
                          "us": {str(p): round(min(v), 1) for p, v in res.items()},
                          "TF": {str(p): round(2 * M * N * K / min(v) / 1e6) for p, v in res.items()}}), flush=True)
        del ops
    for Mw, Nw in ((8192, 1024), (1024, 4096), (3072, 1024)):
        s = asm_wgrad_splits(M, Mw, Nw)
        A0, B0 = rnd(M, Mw), rnd(M, Nw)
        ops = {p: (padded(A0, p), padded(B0, p)) for p in pads}
        del A0, B0
        res = {p: [] for p in pads}
        for _ in range(a.rounds):
            for p in pads:
                A, B = ops[p]
                out = torch.empty(Mw, Nw, device="cuda", dtype=torch.float32)
                res[p].append(timed(lambda: C().asm_wgrad_(out, A, B, s, False)))
        print(json.dumps({"kind": "tn", "Ktot": M, "M": Mw, "N": Nw, "splits": s,
                          "us": {str(p): round(min(v), 1) for p, v in res.items()},
                          "TF": {str(p): round(2 * M * Mw * Nw / min(v) / 1e6) for p, v in res.items()}}), flush=True)
        del ops


if __name__ == "__main__":
    main()
