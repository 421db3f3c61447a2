"""Decode-step projection GEMMs (M = batch) at the reference model's shapes: the skinny MFMA kernels
(csrc/kernels/skinny.hip, epilogue fused) vs hipBLASLt via F.linear (+ the separate epilogue kernel).

Each op is captured 50x into a hipGraph (launch overhead excluded, as in the decode graph) and timed
with events; weights rotate over 5 copies like the reference model's 5 shared blocks. Prints one
JSON line per shape.

    python benchmarks/bench_skinny.py --batch 64
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))


def graph_time(fn, reps=50, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn(0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for r in range(reps):
            fn(r)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / (iters * reps)  # us per call


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--sweep", action="store_true", help="time every (column blocks per wave, waves) shape")
    ap.add_argument("--ablate", action="store_true", help="also time with the X / W / both loads skipped")
    args = ap.parse_args()
    from dalle_amd.ops.hip_ops import C
    dev = torch.device("cuda")
    M, d = args.batch, args.dim
    nw = 5
    cnt = torch.zeros(8192, dtype=torch.int32, device=dev)
    x = torch.randn(M, 4 * d, device=dev).bfloat16()
    resid = torch.randn(M, d, device=dev)
    scale = torch.rand(d, device=dev)
    cos = torch.rand(2048, 64, device=dev)
    sin = torch.rand(2048, 64, device=dev)
    H = d // 64
    q = torch.zeros(M * H, 64, dtype=torch.bfloat16, device=dev)
    kc = torch.zeros(M * H, 1280, 64, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    pos = torch.tensor(300, dtype=torch.int32, device=dev)

    def weights(n, k):
        return [(0.02 * torch.randn(n, k, device=dev)).bfloat16() for _ in range(nw)], \
               [torch.randn(n, device=dev).bfloat16() for _ in range(nw)]

    cases = []
    wq, _ = weights(3 * d, d)
    cases.append(("qkv_rope", 3 * d, d, wq[0].numel() * 2,
                  lambda r: C().skinny_qkv_rope_(x[:, :d], wq[r % nw], cos, sin, q, kc, vc, pos, H, 0.125, cnt),
                  lambda r: C().decode_rope_(F.linear(x[:, :d], wq[r % nw]), cos, sin, q, kc, vc, pos, H, 0.125)))
    wo, bo = weights(d, d)
    cases.append(("out_resid", d, d, wo[0].numel() * 2,
                  lambda r: C().skinny_residual_(resid, x[:, :d], wo[r % nw], bo[r % nw], scale, cnt),
                  lambda r: C().scale_residual_(resid, F.linear(x[:, :d], wo[r % nw], bo[r % nw]), scale)))
    w1, b1 = weights(8 * d, d)
    cases.append(("ff1_geglu", 8 * d, d, w1[0].numel() * 2,
                  lambda r: C().skinny_geglu(x[:, :d], w1[r % nw], b1[r % nw], cnt),
                  lambda r: C().geglu_fwd(F.linear(x[:, :d], w1[r % nw], b1[r % nw]))))
    w2, b2 = weights(d, 4 * d)
    cases.append(("ff2_resid", d, 4 * d, w2[0].numel() * 2,
                  lambda r: C().skinny_residual_(resid, x, w2[r % nw], b2[r % nw], scale, cnt),
                  lambda r: C().scale_residual_(resid, F.linear(x, w2[r % nw], b2[r % nw]), scale)))
    wh, bh = weights(8192, d)
    cases.append(("head_f32", 8192, d, wh[0].numel() * 2,
                  lambda r: C().skinny_linear(x[:, :d], wh[r % nw], bh[r % nw], True, cnt),
                  lambda r: F.linear(x[:, :d], wh[r % nw], bh[r % nw]).float()))
    xs = x[:, :d].contiguous()
    for name, n, k, wbytes, ours, lib in cases:
        G = 2 if name == "ff1_geglu" else 1
        nout = n // G
        t_lib = graph_time(lib)
        configs = [(0, 0, 0, 0)]
        if args.sweep:
            configs += [(nbv, wk, ks, 0) for nbv in (1, 2) for wk in (2, 4, 8) for ks in (1, 2, 4)]
        if args.ablate:
            configs += [(0, 0, 0, 1), (0, 0, 0, 2), (0, 0, 0, 3), (0, 0, 0, 4), (0, 0, 0, 5)]
        seen = set()
        for nbv, wk, ks, dbg in configs:
            C().skinny_force_config(nbv, wk, ks, dbg)
            shape = tuple(C().skinny_shape_info(M, nout, k, G)) + (dbg,)
            if shape in seen:
                continue
            seen.add(shape)
            t_ours = graph_time(ours)
            print(json.dumps({"op": name, "M": M, "N": n, "K": k, "auto": nbv == 0, "nbv_wk_ks_steps_dbg": shape,
                              "skinny_us": round(t_ours, 2), "hipblaslt_us": round(t_lib, 2),
                              "speedup": round(t_lib / t_ours, 2), "skinny_TBps": round(wbytes / t_ours / 1e6, 2)}), flush=True)
        C().skinny_force_config(0, 0, 0, 0)
    del xs


if __name__ == "__main__":
    main()
