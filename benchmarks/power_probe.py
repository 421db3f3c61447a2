"""Board power and shader clock while a GEMM runs back to back: is the long-K assembly GEMM (or its no-DMA
diagnostic build) running at the power limit, with the clock -- not the schedule -- setting its speed?

    python benchmarks/power_probe.py [--seconds 6]

Each variant loops for --seconds while a sampler thread reads `rocm-smi --showpower --showclocks --json`
about once a second (a child process; read-only). Prints per variant: microseconds per GEMM and the
sampled power / sclk values; the first raw sample goes to gpurun_out/power_probe_raw.json."""
import argparse
import json
import os
import re
import subprocess
import sys
import threading
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)
from bench_asm_gemm import Module, gemm_args  # noqa: E402
from dalle_amd.ops.hip_ops import C  # noqa: E402


def smi():
    try:
        return subprocess.run(["rocm-smi", "--showpower", "--showclocks", "--json"], capture_output=True, text=True,
                              timeout=20).stdout
    except Exception as e:  # noqa: BLE001
        return json.dumps({"error": str(e)})


def numbers(raw: str):
    """(power W, sclk MHz) from one rocm-smi JSON sample (keys vary between versions: match by name)."""
    try:
        d = json.loads(raw)
    except ValueError:
        return None, None
    pw = sc = None
    for card in d.values():
        if not isinstance(card, dict):
            continue
        for k, v in card.items():
            kl = k.lower()
            m = re.search(r"[\d.]+", str(v))
            if m is None:
                continue
            if "power" in kl and pw is None:
                pw = float(m.group(0))
            if "sclk" in kl and sc is None:
                sc = float(re.findall(r"[\d.]+", str(v))[-1]) if "mhz" in str(v).lower() else float(m.group(0))
    return pw, sc


def run(name, fn, seconds, raw_out):
    samples, stop = [], threading.Event()

    def sampler():
        while not stop.is_set():
            raw = smi()
            if raw_out is not None and not os.path.exists(raw_out):
                with open(raw_out, "w") as f:
                    f.write(raw)
            samples.append(numbers(raw))
            time.sleep(0.7)

    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    th = threading.Thread(target=sampler, daemon=True)
    th.start()
    t0, n = time.time(), 0
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    while time.time() - t0 < seconds:
        for _ in range(10):
            fn()
        n += 10
        torch.cuda.synchronize()
    ev1.record()
    torch.cuda.synchronize()
    stop.set()
    th.join(timeout=30)
    us = ev0.elapsed_time(ev1) * 1000.0 / n
    good = [s for s in samples[1:] if s[0] is not None or s[1] is not None]
    print(json.dumps({"variant": name, "us": round(us, 1), "samples": good}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    a = ap.parse_args()
    os.makedirs("gpurun_out", exist_ok=True)
    raw = "gpurun_out/power_probe_raw.json"
    diag = Module(os.path.join(HERE, "..", "dalle_amd", "gemm_diag_gfx950.hsaco"))
    M, N, K = 163840, 1024, 8192
    A = torch.randn(M, K, device="cuda", dtype=torch.bfloat16) * 0.02
    B = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    Cm = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    args = gemm_args(A, B, Cm)
    run("idle_sleep", lambda: time.sleep(0.05), min(a.seconds, 3.0), raw)
    run("asm_nt_K8192", lambda: C().asm_gemm(A, B, None, Cm), a.seconds, None)
    run("asm_nt_K8192_nodma", lambda: diag.launch("dalle_gemm_diag_nodma", 256, args), a.seconds, None)
    run("asm_nt_K8192_serp", lambda: diag.launch("dalle_gemm_diag_serp", 256, args), a.seconds, None)
    run("asm_nt_K8192_ant", lambda: diag.launch("dalle_gemm_diag_ant", 256, args), a.seconds, None)
    run("asm_nt_K8192_abnt", lambda: diag.launch("dalle_gemm_diag_abnt", 256, args), a.seconds, None)
    run("asm_nt_K8192_again", lambda: C().asm_gemm(A, B, None, Cm), a.seconds, None)
    run("hipblaslt_K8192", lambda: torch.mm(A, B.t(), out=Cm), a.seconds, None)
    Z = torch.zeros_like(A)
    Zb = torch.zeros_like(B)
    run("asm_nt_K8192_zeros", lambda: C().asm_gemm(Z, Zb, None, Cm), a.seconds, None)


if __name__ == "__main__":
    main()
