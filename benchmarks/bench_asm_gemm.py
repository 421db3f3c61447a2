"""Standalone check + A/B of the generated assembly GEMM (csrc/asm/gen_gemm.py) against hipBLASLt.

Loads the code object through the HIP module API (ctypes), so it needs no extension build:

    python benchmarks/bench_asm_gemm.py [--hsaco path] [--check-only] [--shapes M:N:K,...]

Prints one JSON line per shape: microseconds and TF/s of hipBLASLt (torch.matmul) and of each kernel,
interleaved in one process on the same random operands (rule: A/B in one process).
"""
import argparse
import ctypes
import json
import os
import struct
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


class Module:
    def __init__(self, path):
        self.hip = ctypes.CDLL("libamdhip64.so")
        data = open(path, "rb").read()
        self._buf = ctypes.create_string_buffer(data, len(data))
        self.mod = ctypes.c_void_p()
        err = self.hip.hipModuleLoadData(ctypes.byref(self.mod), self._buf)
        assert err == 0, f"hipModuleLoadData: {err}"
        self.funcs = {}

    def func(self, name):
        if name not in self.funcs:
            f = ctypes.c_void_p()
            err = self.hip.hipModuleGetFunction(ctypes.byref(f), self.mod, name.encode())
            assert err == 0, f"hipModuleGetFunction({name}): {err}"
            self.funcs[name] = f
        return self.funcs[name]

    def launch(self, name, grid, args: bytes, stream=None):
        f = self.func(name)
        buf = ctypes.create_string_buffer(args, len(args))
        size = ctypes.c_size_t(len(args))
        extra = (ctypes.c_void_p * 5)(1, ctypes.cast(buf, ctypes.c_void_p), 2,
                                      ctypes.cast(ctypes.byref(size), ctypes.c_void_p), 3)
        st = ctypes.c_void_p(stream if stream is not None else torch.cuda.current_stream().cuda_stream)
        err = self.hip.hipModuleLaunchKernel(f, grid, 1, 1, 256, 1, 1, 0, st, None, extra)
        assert err == 0, f"hipModuleLaunchKernel: {err}"


def gemm_args(A, B, C, aux0=None, grid=256):
    M, K = A.shape
    N = B.shape[0]
    assert M % 256 == 0 and N % 256 == 0 and K % 128 == 0 and K >= 256
    assert A.stride(1) == 1 and B.stride(1) == 1 and C.stride(1) == 1
    tiles_n = N // 256
    nt = (M // 256) * tiles_n
    ptrs = [A.data_ptr(), B.data_ptr(), C.data_ptr(), aux0.data_ptr() if aux0 is not None else 0, 0, 0]
    ints = [M, N, K, A.stride(0), B.stride(0), C.stride(0), tiles_n, nt, grid, 0, 0, 0]
    return struct.pack("<6Q16i", *ptrs, *ints, 0, 0, 0, 0)


def run(mod, name, A, B, C, aux0=None, grid=None):
    M, N = A.shape[0], B.shape[0]
    nt = (M // 256) * (N // 256)
    if grid is None:
        grid = min(256, (nt + 7) // 8 * 8)
    mod.launch(name, grid, gemm_args(A, B, C, aux0, grid))


def tn_args(A, B, part, splits):
    Ktot, M = A.shape
    N = B.shape[1]
    units = (M // 256) * (N // 256) * splits
    ptrs = [A.data_ptr(), B.data_ptr(), part.data_ptr(), 0, 0, 0]
    ints = [M, N, Ktot // splits, A.stride(0), B.stride(0), N, N // 256, units, units, 0, 0, 0]
    return units, struct.pack("<6Q16i", *ptrs, *ints, 0, 0, 0, 0)


def run_tn(mod, A, B, part, splits):
    units, args = tn_args(A, B, part, splits)
    mod.launch("dalle_gemm_tn_wgrad", units, args)


def check_tn(mod, shapes):
    ok = True
    for (Ktot, M, N, splits) in shapes:
        torch.manual_seed(Ktot + M + N)
        A = torch.randn(Ktot, M, device="cuda").to(torch.bfloat16)
        B = torch.randn(Ktot, N, device="cuda").to(torch.bfloat16)
        part = torch.full((splits, M, N), float("nan"), device="cuda")
        run_tn(mod, A, B, part, splits)
        torch.cuda.synchronize()
        ref = A.float().t() @ B.float()
        got = part.sum(0)
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        nan = torch.isnan(got).sum().item()
        good = err < 1e-3 and nan == 0
        ok &= good
        print(json.dumps({"check": "tn_wgrad", "Ktot": Ktot, "M": M, "N": N, "splits": splits, "max_rel_err": err,
                          "nan": nan, "ok": good}), flush=True)
    return ok


def bench_tn(mod, shapes, iters=10, rounds=5, diag=None):
    for (Ktot, M, N, splits) in shapes:
        A = torch.rand(Ktot, M, device="cuda").sub_(0.5).to(torch.bfloat16)
        B = torch.rand(Ktot, N, device="cuda").sub_(0.5).to(torch.bfloat16)
        part = torch.empty(splits, M, N, device="cuda")
        out = torch.empty(M, N, device="cuda")
        fns = {
            "hipblaslt_tn": lambda: torch.mm(A.t(), B, out_dtype=torch.float32, out=out),
            "asm_tn": lambda: run_tn(mod, A, B, part, splits),
            "asm_tn+fold": lambda: (run_tn(mod, A, B, part, splits), torch.sum(part, 0, out=out)),
        }
        if diag is not None:
            fns["asm_tn_nodma"] = lambda: diag.launch("dalle_gemm_diag_tn_nodma", *tn_args(A, B, part, splits))
            fns["asm_tn_afirst"] = lambda: diag.launch("dalle_gemm_diag_tn_afirst", *tn_args(A, B, part, splits))
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in fns}
        for _ in range(rounds):
            for k, f in fns.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(iters):
                    f()
                e.record()
                e.synchronize()
                times[k].append(s.elapsed_time(e) * 1000 / iters)
        flop = 2.0 * M * N * Ktot
        us = {k: round(sorted(v)[len(v) // 2], 1) for k, v in times.items()}
        print(json.dumps({"shape": f"TN_K{Ktot}_M{M}_N{N}_s{splits}", "us": us,
                          "TF": {k: round(flop / v / 1e6) for k, v in us.items()}}), flush=True)


def bench_geglu(mod, M=163840, F=4096, K=1024, iters=10, rounds=3, diag=None):
    """FF-in GEMM + fused GEGLU vs the same GEMM with the bias epilogue only (the fusion's extra cost)"""
    x = torch.rand(M, K, device="cuda").sub_(0.5).to(torch.bfloat16)
    w = torch.rand(2 * F, K, device="cuda").sub_(0.5).mul_(0.06).to(torch.bfloat16)
    b = torch.zeros(2 * F, device="cuda")
    a = torch.empty(M, 2 * F, device="cuda", dtype=torch.bfloat16)
    u = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    nt = (M // 256) * (2 * F // 256)
    grid = min(256, (nt + 7) // 8 * 8)
    ptrs = [x.data_ptr(), w.data_ptr(), a.data_ptr(), b.data_ptr(), u.data_ptr(), 0]
    ints = [M, 2 * F, K, K, K, 2 * F, 2 * F // 256, nt, grid, F, 0, 0]
    args = struct.pack("<6Q16i", *ptrs, *ints, 0, 0, 0, 0)
    fns = {"asm_bias": lambda: mod.launch("dalle_gemm_nt_bias", grid, args),
           "asm_geglu": lambda: mod.launch("dalle_gemm_nt_geglu", grid, args)}
    if diag is not None:
        fns["asm_geglu_nowork"] = lambda: diag.launch("dalle_gemm_diag_geglu_nowork", grid, args)
        fns["asm_geglu_adjacent"] = lambda: diag.launch("dalle_gemm_diag_geglu_adjacent", grid, args)

    for f in fns.values():
        f()
    torch.cuda.synchronize()
    times = {k: [] for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                f()
            e.record()
            e.synchronize()
            times[k].append(s.elapsed_time(e) * 1000 / iters)
    us = {k: round(sorted(v)[len(v) // 2], 1) for k, v in times.items()}
    print(json.dumps({"shape": f"GEGLU_M{M}_F{F}_K{K}", "us": us}), flush=True)


def bench_geglu_bwd(mod, M=163840, F=4096, K=1024, iters=10, rounds=3, diag=None):
    """FF-out dgrad + GEGLU backward on the assembly kernel vs the plain GEMM of the same shape (the fused
    backward's extra cost) and the HIP 8-phase kernel it replaces (extension)"""
    dy = torch.rand(M, K, device="cuda").sub_(0.5).to(torch.bfloat16)
    w2t = torch.rand(F, K, device="cuda").sub_(0.5).mul_(0.06).to(torch.bfloat16)
    h = torch.randn(M, 2 * F, device="cuda").to(torch.bfloat16)
    dh = torch.empty_like(h)
    du = torch.empty(M, F, device="cuda", dtype=torch.bfloat16)
    part = torch.empty(M // 128, 2 * F, device="cuda")
    nt = (M // 256) * (F // 256)
    grid = min(256, (nt + 7) // 8 * 8)
    ptrs = [dy.data_ptr(), w2t.data_ptr(), dh.data_ptr(), h.data_ptr(), part.data_ptr(), 0]
    args = struct.pack("<6Q16i", *ptrs, M, F, K, K, K, 2 * F, F // 256, nt, grid, F, 0, 0, 0, 0, 0, 0)
    fns = {"asm_plain": lambda: run(mod, "dalle_gemm_nt_plain", dy, w2t, du),
           "asm_geglu_bwd": lambda: mod.launch("dalle_gemm_nt_geglu_bwd", grid, args)}
    if diag is not None:
        for v in ("novalu", "nomem"):
            fns[f"asm_gbwd_{v}"] = (lambda v=v: diag.launch(f"dalle_gemm_diag_gbwd_{v}", grid, args))
    try:
        sys.path.insert(0, os.path.join(HERE, ".."))
        from dalle_amd.ops.ext import load_extension
        C = load_extension(required=True)
        fns["hip_8ph"] = lambda: C.ff_dgrad_geglu(dy, w2t, h, None)
        fns["ext_asm"] = lambda: C.asm_ff_dgrad_geglu(dy, w2t, h, None)
    except Exception as ex:   # extension not built: the code-object kernels only
        print(json.dumps({"note": f"extension not loaded: {ex}"}))
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    times = {k: [] for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(iters):
                f()
            e.record()
            e.synchronize()
            times[k].append(s.elapsed_time(e) * 1000 / iters)
    flop = 2.0 * M * F * K
    us = {k: round(sorted(v)[len(v) // 2], 1) for k, v in times.items()}
    print(json.dumps({"shape": f"GEGLU_BWD_M{M}_F{F}_K{K}", "us": us,
                      "TF": {k: round(flop / v / 1e6) for k, v in us.items()}}), flush=True)


def check(mod, shapes):
    ok = True
    for (M, N, K) in shapes:
        torch.manual_seed(M + N + K)
        A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
        bias = torch.randn(N, device="cuda")
        ref = A.float() @ B.float().t()
        for name, aux in (("dalle_gemm_nt_plain", None), ("dalle_gemm_nt_bias", bias)):
            C = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
            run(mod, name, A, B, C, aux)
            torch.cuda.synchronize()
            r = ref + (bias if aux is not None else 0)
            err = ((C.float() - r).abs().max() / r.abs().max()).item()
            nan = torch.isnan(C.float()).sum().item()
            good = err < 1e-2 and nan == 0
            ok &= good
            print(json.dumps({"check": name, "M": M, "N": N, "K": K, "max_rel_err": err, "nan": nan, "ok": good}),
                  flush=True)
    return ok


def bench(mod, shapes, iters=20, diag=None, rounds=5):
    for (M, N, K) in shapes:
        A = torch.rand(M, K, device="cuda").sub_(0.5).to(torch.bfloat16)
        B = torch.rand(N, K, device="cuda").sub_(0.5).to(torch.bfloat16)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fns = {
            "hipblaslt": lambda: torch.mm(A, B.t(), out=C),
            "asm_plain": lambda: run(mod, "dalle_gemm_nt_plain", A, B, C),
        }
        if diag is not None:
            for v in ("noepi", "nodma", "split", "nostagger", "nostore", "nopack", "defer4", "afirst", "serp", "ant", "abnt"):
                fns[f"asm_{v}"] = (lambda v=v: run(diag, f"dalle_gemm_diag_{v}", A, B, C))
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in fns}
        for _ in range(rounds):   # interleaved rounds
            for k, f in fns.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(iters):
                    f()
                e.record()
                e.synchronize()
                times[k].append(s.elapsed_time(e) * 1000 / iters)
        flop = 2.0 * M * N * K
        us = {k: round(sorted(v)[len(v) // 2], 1) for k, v in times.items()}
        print(json.dumps({"shape": f"M{M}_N{N}_K{K}", "us": us,
                          "TF": {k: round(flop / v / 1e6) for k, v in us.items()}}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hsaco", default=os.path.join(HERE, "..", "dalle_amd", "gemm_gfx950.hsaco"))
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--diag", action="store_true", help="also time the measurement-only variants")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tn", action="store_true", help="also time the weight-gradient (TN) kernel")
    ap.add_argument("--geglu", action="store_true", help="also time the fused FF-in + GEGLU kernel")
    ap.add_argument("--geglu-bwd", action="store_true", help="also time the FF-out dgrad + GEGLU backward kernel")
    ap.add_argument("--skip-plain", action="store_true", help="skip the plain-GEMM shape sweep")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shapes", default="163840:1024:1024,163840:3072:1024,163840:4096:1024,163840:8192:1024,"
                                        "163840:1024:4096,163840:1024:8192,163840:1024:3072")
    a = ap.parse_args()
    mod = Module(a.hsaco)
    ok = check(mod, [(256, 256, 256), (512, 768, 384), (1024, 512, 1024), (2560, 3072, 1024), (4096, 1024, 4096),
                     (25600, 768, 512), (9 * 256, 1024, 512), (17 * 256, 256, 512), (259 * 256, 3 * 256, 512)])
    ok &= check_tn(mod, [(2048, 256, 256, 1), (4096, 512, 768, 2), (8192, 1024, 1024, 4), (16384, 3072, 1024, 16),
                         (3 * 8192, 768, 512, 3)])
    if not ok:
        sys.exit(1)
    if a.check_only:
        return
    if a.geglu:
        bench_geglu(mod, rounds=a.rounds,
                    diag=Module(os.path.join(HERE, "..", "dalle_amd", "gemm_diag_gfx950.hsaco")) if a.diag else None)
    if a.geglu_bwd:
        bench_geglu_bwd(mod, rounds=a.rounds,
                        diag=Module(os.path.join(HERE, "..", "dalle_amd", "gemm_diag_gfx950.hsaco")) if a.diag else None)
    if a.tn:
        bench_tn(mod, [(163840, 1024, 1024, 16), (163840, 3072, 1024, 16), (163840, 8192, 1024, 2),
                       (163840, 1024, 4096, 4)], rounds=a.rounds,
                 diag=Module(os.path.join(HERE, "..", "dalle_amd", "gemm_diag_gfx950.hsaco")) if a.diag else None)
    if a.skip_plain:
        return
    shapes = [tuple(int(x) for x in s.split(":")) for s in a.shapes.split(",")]
    diag = Module(os.path.join(HERE, "..", "dalle_amd", "gemm_diag_gfx950.hsaco")) if a.diag else None
    bench(mod, shapes, iters=a.iters, diag=diag, rounds=a.rounds)


if __name__ == "__main__":
    main()
