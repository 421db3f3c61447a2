"""Where the assembly QKV + rotary kernel disagrees with the unfused path (projection, then rope_fwd): per
(part, head) the storage rows whose error exceeds 1e-2 of the max, as row ranges; also a plain asm GEMM of the
same operands against the projection (isolates the GEMM from the rotation / scatter)."""
import torch

from dalle_amd.models.patterns import AttnGeometry
from dalle_amd.ops.ext import load_extension
from dalle_amd.ops.hip_ops import _cs3_from_tables, _rope_tables


def ranges(idx):
    out, start, prev = [], None, None
    for i in idx:
        if start is None:
            start = prev = i
        elif i == prev + 1:
            prev = i
        else:
            out.append((start, prev))
            start = prev = i
    if start is not None:
        out.append((start, prev))
    return out


def main():
    C = load_extension(required=True)
    dev = torch.device("cuda:0")
    torch.manual_seed(7)
    T, S, H, B = 257, 32, 16, 2
    n = T + S * S - 1
    geom = AttnGeometry(T, S, 5)
    h = torch.randn(B * n, 1024, device=dev).to(torch.bfloat16)
    w = (torch.randn(3 * H * 64, 1024, device=dev) * 0.03).to(torch.bfloat16)
    cos, sin = _rope_tables(geom, 64, dev)
    ref_proj = (h.float() @ w.float().t())
    g = C.asm_gemm(h, w, None, None).float()
    print("plain asm gemm rel err", ((g - ref_proj).abs().max() / ref_proj.abs().max()).item())
    cs3 = _cs3_from_tables(cos, sin, 0.125)
    print("cs3", tuple(cs3.shape), "cos", tuple(cos.shape))
    for col in (False, True):
        q, k, v = C.asm_qkv_rope(h, w, cs3, T, S, H, n, col)
        torch.cuda.synchronize()
        qkv = ref_proj.to(torch.bfloat16).view(B, n, -1)
        q2, k2, v2 = C.rope_fwd(qkv, cos, sin, T, S, H, col, 0.125)
        for name, a, b in (("q", q, q2), ("k", k, k2), ("v", v, v2)):
            d = (a.float() - b.float()).abs()
            scale = b.float().abs().max().item()
            bad = (d.amax(-1) > 1e-2 * scale)            # (B H, Np)
            print(f"col={col} {name}: max rel err {d.max().item() / scale:.3e}, bad rows {int(bad.sum())} of {bad.numel()}")
            shown = 0
            for bh in range(bad.shape[0]):
                rows = torch.nonzero(bad[bh]).flatten().tolist()
                if rows and shown < 12:
                    r = ranges(rows)
                    zero = int((a[bh][bad[bh]].float().abs().amax(-1) == 0).sum())
                    print(f"   head {bh}: {len(rows)} bad rows (zero: {zero}) {r[:8]}{' ...' if len(r) > 8 else ''}")
                    shown += 1


if __name__ == "__main__":
    main()
