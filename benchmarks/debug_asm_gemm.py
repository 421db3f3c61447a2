"""Diagnostics for the assembly GEMM: structured operands, a sentinel-filled output, and a map of which
16 x 16 output blocks are unwritten / wrong (used while bringing the generator up)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_asm_gemm import Module, run  # noqa: E402


def main():
    mod = Module(os.path.join(os.path.dirname(__file__), "..", "dalle_amd", "gemm_gfx950.hsaco"))
    M = N = K = 256
    dev = "cuda"
    cases = {
        "ones": (torch.ones(M, K), torch.ones(N, K)),
        "rowid": (torch.arange(M).float().view(-1, 1).expand(M, K) / 64, torch.ones(N, K) / K),
        "colid": (torch.ones(M, K) / K, torch.arange(N).float().view(-1, 1).expand(N, K) / 64),
        "kid": (torch.ones(M, K), (torch.arange(K).float().view(1, -1).expand(N, K) % 8)),
        "randn": (torch.randn(M, K), torch.randn(N, K)),
    }
    for name, (a, b) in list(cases.items()) + [("ones_again", cases["ones"])]:
        A = a.to(dev).to(torch.bfloat16).contiguous()
        B = b.to(dev).to(torch.bfloat16).contiguous()
        C = torch.full((M, N), 12345.0, device=dev, dtype=torch.bfloat16)
        run(mod, "dalle_gemm_nt_plain", A, B, C)
        torch.cuda.synchronize()
        ref = A.float() @ B.float().t()
        c = C.float()
        unwritten = (c == 12352.0)
        nan = torch.isnan(c)
        bad = ~(torch.isclose(c, ref, rtol=2e-2, atol=1e-1)) & ~unwritten & ~nan
        blk = lambda t: t.view(64, 4, 32, 8).any(3).any(1).int()  # noqa: E731 (4-row x 8-col blocks)
        out = {"case": name, "unwritten": int(unwritten.sum()), "nan": int(nan.sum()), "bad": int(bad.sum())}
        print(json.dumps(out), flush=True)
        for what, t in (("unwritten", unwritten), ("nan", nan), ("bad", bad)):
            if t.any():
                m = blk(t)
                print(what, "blocks (64x32 grid of 4-row x 8-col blocks):")
                for r in range(64):
                    print("  " + "".join("#" if v else "." for v in m[r].tolist()))
        if name in ("ones", "rowid", "colid", "kid"):
            print("C[0:4,0:12]", [[round(x, 2) for x in row] for row in c[:4, :12].tolist()])
            print("ref[0:4,0:12]", [[round(x, 2) for x in row] for row in ref[:4, :12].tolist()])
            print("C[16:18,128:136]", [[round(x, 2) for x in row] for row in c[16:18, 128:136].tolist()])


if __name__ == "__main__":
    main()
