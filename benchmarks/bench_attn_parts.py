#!/usr/bin/env python3
"""Attention kernels one by one at the bench24 geometry (T = 257, 32 x 32 image, 16 heads x 64) and the
training micro-batch (default 128; argv[1]): forward (attn_fwd) and the rotary-fused backward
(attn_bwd_rope: dQ [+ fused local dK/dV] + text dK/dV [+ image dK/dV]), per pattern, device-timed
(median of rounds). One JSON line per pattern; with ``--check`` every output is also compared against
the PyTorch reference path on a small batch first."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.models.patterns import AttnGeometry, PATTERN_IDS  # noqa: E402
from dalle_amd.ops import hip_ops  # noqa: E402


def timed(fn, rounds=7):
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 128
    C = hip_ops.C()
    dev = torch.device("cuda")
    T, S, H, D = 257, 32, 16, 1024
    n = T + S * S - 1
    geom = AttnGeometry(T, S, 5)
    torch.manual_seed(0)
    h = torch.randn(B * n, D, device=dev).bfloat16()
    w = (0.03 * torch.randn(3 * H * 64, D, device=dev)).bfloat16()
    cos, sin = hip_ops._rope_tables(geom, 64, dev)
    cs = hip_ops.rope_cs_table(geom, 64, dev)
    res = {}
    for pat in ("axial_row", "axial_col", "conv_like"):
        col = pat == "axial_col"
        pid = PATTERN_IDS[pat]
        q, k, v = C.qkv_rope_pt(h, w, cs, T, S, H, n, col, 0.125)
        out, lse = C.attn_fwd(q, k, v, B, T, S, n, geom.kernel_size, H, pid)
        do = (0.1 * torch.randn_like(out)).contiguous()
        t_f = timed(lambda: C.attn_fwd(q, k, v, B, T, S, n, geom.kernel_size, H, pid))
        t_b = timed(lambda: C.attn_bwd_rope(q, k, v, out, do, lse, cos, sin, B, T, S, n, geom.kernel_size, H, pid, 0.125))
        res[pat] = {"fwd_us": t_f, "bwd_us": t_b}
        print(json.dumps({"pattern": pat, "B": B, "fwd_us": t_f, "bwd_us": t_b}), flush=True)
        del q, k, v, out, lse, do
    # the bench24 layer mix: 23 layers cycling row, col, row, row + 1 conv_like
    mix = {"axial_row": 17, "axial_col": 6, "conv_like": 1}
    per_step = sum(mix[p] * (res[p]["fwd_us"] + res[p]["bwd_us"]) for p in mix) / 1e3
    print(json.dumps({"bench24_attention_ms_per_step": round(per_step, 2), "per_layer_us": round(per_step * 1e3 / 24, 1)}), flush=True)


if __name__ == "__main__":
    main()
