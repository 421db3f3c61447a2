"""A/B of GEMM builds under the board power limit: each variant runs back to back for --seconds (the power
controller settles within ~1 s), only the last --seconds - 1 s are timed, and the variants alternate for
--rounds rounds (A B A B ...), so neither gets the clock headroom another variant's cooler run leaves behind
(which biases the short interleaved timings of bench_asm_gemm.py towards whichever variant follows a cool one).

    python benchmarks/ab_sustained.py [--seconds 3] [--rounds 3]

Prints one JSON line per comparison: per-variant median microseconds and the B / A ratio."""
import argparse
import json
import os
import statistics
import struct
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)
from bench_asm_gemm import Module, gemm_args, tn_args  # noqa: E402


def sustained(fn, seconds):
    t_end = time.time() + seconds
    t_meas = t_end - (seconds - 1.0)
    n, started = 0, False
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    while True:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        now = time.time()
        if not started and now >= t_meas:
            e0.record()
            started, n = True, 0
            continue
        if started:
            n += 5
            if now >= t_end:
                break
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / n


def compare(name, fa, fb, seconds, rounds):
    ta, tb = [], []
    for _ in range(rounds):
        ta.append(sustained(fa, seconds))
        tb.append(sustained(fb, seconds))
    a, b = statistics.median(ta), statistics.median(tb)
    print(json.dumps({"cmp": name, "a_us": round(a, 1), "b_us": round(b, 1), "b_over_a": round(b / a, 4),
                      "a_all": [round(x, 1) for x in ta], "b_all": [round(x, 1) for x in tb]}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--suite", default="order", choices=["order", "nosplit", "plain", "fused", "splits"])
    ap.add_argument("--variants", default="nostagger,defer4,l2store", help="suite plain: diag builds vs production")
    ap.add_argument("--shapes", default="1024:1024,8192:1024,1024:8192", help="suite plain: N:K at M = 163840")
    a = ap.parse_args()
    prod = Module(os.path.join(HERE, "..", "dalle_amd", "gemm_gfx950.hsaco"))
    diag = Module(os.path.join(HERE, "..", "dalle_amd", "gemm_diag_gfx950.hsaco"))
    M = 163840
    if a.suite == "splits":  # weight-grad split count, kernel + deterministic fold (the extension's asm_wgrad_)
        from dalle_amd.ops.hip_ops import C
        for Mw, Nw, sa, sb in ((3072, 1024, 16, 5), (3072, 1024, 16, 10), (1024, 1024, 16, 10), (1024, 4096, 4, 5)):
            A = torch.randn(M, Mw, device="cuda", dtype=torch.bfloat16) * 0.02
            B = torch.randn(M, Nw, device="cuda", dtype=torch.bfloat16) * 0.02
            out = torch.zeros(Mw, Nw, device="cuda")
            compare(f"wgrad {Mw}x{Nw}: s{sa} vs s{sb}", lambda: C().asm_wgrad_(out, A, B, sa, True),
                    lambda: C().asm_wgrad_(out, A, B, sb, True), a.seconds, a.rounds)
            del A, B, out
        return
    if a.suite == "fused":  # split release (production) vs one release barrier: TN weight grad, FF-in + GEGLU, GEGLU bwd
        for Mw, Nw, sp in ((8192, 1024, 2), (1024, 4096, 4), (3072, 1024, 16)):
            A = torch.randn(M, Mw, device="cuda", dtype=torch.bfloat16) * 0.02
            B = torch.randn(M, Nw, device="cuda", dtype=torch.bfloat16) * 0.02
            part = torch.empty(sp, Mw, Nw, device="cuda")
            units, args = tn_args(A, B, part, sp)
            compare(f"tn {Mw}x{Nw} s{sp}: production vs tn_onebar",
                    lambda: prod.launch("dalle_gemm_tn_wgrad", units, args),
                    lambda: diag.launch("dalle_gemm_diag_tn_onebar", units, args), a.seconds, a.rounds)
            del A, B, part
        F, K = 4096, 1024
        x = torch.rand(M, K, device="cuda").sub_(0.5).to(torch.bfloat16)
        w = torch.rand(2 * F, K, device="cuda").sub_(0.5).mul_(0.06).to(torch.bfloat16)
        b = torch.zeros(2 * F, device="cuda")
        av = torch.empty(M, 2 * F, device="cuda", dtype=torch.bfloat16)
        u = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
        nt = (M // 256) * (2 * F // 256)
        grid = min(256, (nt + 7) // 8 * 8)
        args = struct.pack("<6Q16i", x.data_ptr(), w.data_ptr(), av.data_ptr(), b.data_ptr(), u.data_ptr(), 0,
                           M, 2 * F, K, K, K, 2 * F, 2 * F // 256, nt, grid, F, 0, 0, 0, 0, 0, 0)
        compare("geglu F4096: production vs nosplit", lambda: prod.launch("dalle_gemm_nt_geglu", grid, args),
                lambda: diag.launch("dalle_gemm_diag_geglu_nosplit", grid, args), a.seconds, a.rounds)
        del x, w, av, u
        dy = torch.rand(M, K, device="cuda").sub_(0.5).to(torch.bfloat16)
        w2t = torch.rand(F, K, device="cuda").sub_(0.5).mul_(0.06).to(torch.bfloat16)
        h = torch.randn(M, 2 * F, device="cuda").to(torch.bfloat16)
        dh = torch.empty_like(h)
        part = torch.empty(M // 128, 2 * F, device="cuda")
        nt = (M // 256) * (F // 256)
        grid = min(256, (nt + 7) // 8 * 8)
        args = struct.pack("<6Q16i", dy.data_ptr(), w2t.data_ptr(), dh.data_ptr(), h.data_ptr(), part.data_ptr(), 0,
                           M, F, K, K, K, 2 * F, F // 256, nt, grid, F, 0, 0, 0, 0, 0, 0)
        compare("geglu_bwd F4096: production vs nosplit", lambda: prod.launch("dalle_gemm_nt_geglu_bwd", grid, args),
                lambda: diag.launch("dalle_gemm_diag_gbwd_nosplit", grid, args), a.seconds, a.rounds)
        return
    if a.suite == "plain":  # production plain kernel vs each named diagnostic build
        for sh in a.shapes.split(","):
            N, K = (int(x) for x in sh.split(":"))
            A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16) * 0.02
            B = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            Cm = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            args = gemm_args(A, B, Cm)
            for v in a.variants.split(","):
                compare(f"nt N{N} K{K}: production vs {v}", lambda: prod.launch("dalle_gemm_nt_plain", 256, args),
                        lambda v=v: diag.launch(f"dalle_gemm_diag_{v}", 256, args), a.seconds, a.rounds)
            del A, B, Cm
        return
    if a.suite == "nosplit":  # every plain shape of the step: one stage-release barrier (prod) vs the split release
        for N, K in ((1024, 1024), (3072, 1024), (1024, 3072), (1024, 4096), (8192, 1024), (1024, 8192)):
            A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16) * 0.02
            B = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            Cm = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            args = gemm_args(A, B, Cm)
            compare(f"nt N{N} K{K}: one release barrier (prod) vs split release",
                    lambda: prod.launch("dalle_gemm_nt_plain", 256, args),
                    lambda: diag.launch("dalle_gemm_diag_split", 256, args), a.seconds, a.rounds)
            del A, B, Cm
        return
    for Mw, Nw, s in ((8192, 1024, 2), (1024, 4096, 4)):
        A = torch.randn(M, Mw, device="cuda", dtype=torch.bfloat16) * 0.02
        B = torch.randn(M, Nw, device="cuda", dtype=torch.bfloat16) * 0.02
        part = torch.empty(s, Mw, Nw, device="cuda")
        units, args = tn_args(A, B, part, s)
        compare(f"tn {Mw}x{Nw} s{s}: B-first (prod) vs A-first",
                lambda: prod.launch("dalle_gemm_tn_wgrad", units, args),
                lambda: diag.launch("dalle_gemm_diag_tn_afirst", units, args), a.seconds, a.rounds)
        del A, B, part
    for N, K in ((1024, 8192), (8192, 1024)):
        A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16) * 0.02
        B = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        Cm = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        args = gemm_args(A, B, Cm)
        compare(f"nt N{N} K{K}: one release barrier (prod) vs split release",
                lambda: prod.launch("dalle_gemm_nt_plain", 256, args),
                lambda: diag.launch("dalle_gemm_diag_split", 256, args), a.seconds, a.rounds)
        compare(f"nt N{N} K{K}: B-first (prod) vs A-first",
                lambda: prod.launch("dalle_gemm_nt_plain", 256, args),
                lambda: diag.launch("dalle_gemm_diag_afirst", 256, args), a.seconds, a.rounds)
        del A, B, Cm


if __name__ == "__main__":
    main()
