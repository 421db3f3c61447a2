#!/usr/bin/env python3
"""One attention backward (attn_bwd_rope) at the bench24 geometry, repeated N times -- a short program for
rocprofv3 PMC passes over the attention backward kernels alone (argv: pattern [axial_row], reps [5], B [128])."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.models.patterns import AttnGeometry, PATTERN_IDS  # noqa: E402
from dalle_amd.ops import hip_ops  # noqa: E402

pat = sys.argv[1] if len(sys.argv) > 1 else "axial_row"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
B = int(sys.argv[3]) if len(sys.argv) > 3 else 128
C = hip_ops.C()
dev = torch.device("cuda")
T, S, H, D = 257, 32, 16, 1024
n = T + S * S - 1
geom = AttnGeometry(T, S, 5)
torch.manual_seed(0)
h = torch.randn(B * n, D, device=dev).bfloat16()
w = (0.03 * torch.randn(3 * H * 64, D, device=dev)).bfloat16()
cos, sin = hip_ops._rope_tables(geom, 64, dev)
col = pat == "axial_col"
pid = PATTERN_IDS[pat]
q, k, v = C.asm_qkv_rope(h, w, hip_ops._cs3_from_tables(cos, sin, 0.125), T, S, H, n, col)
out, lse = C.attn_fwd(q, k, v, B, T, S, n, geom.kernel_size, H, pid)
do = (0.1 * torch.randn_like(out)).contiguous()
rf = hip_ops._rot_freqs(dev)
for _ in range(reps):
    C.attn_bwd_rope(q, k, v, out, do, lse, cos, sin, B, T, S, n, geom.kernel_size, H, pid, 0.125, *rf)
torch.cuda.synchronize()
print("ok")
