#!/usr/bin/env python3
"""K20: VQGAN f8 decoder (the LAION vqgan_gumbel_f8 geometry: 32x32 codes -> 256x256 RGB) on the HIP
kernels vs the PyTorch (MIOpen) decoder, batch 64 by default. One JSON line: ms per batch, images/s,
executed TFLOP/s of the 3x3 convolutions, max |HIP - torch| over the batch."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dalle_amd.models.vqgan import VQGanVAE  # noqa: E402


def conv_flops(dec, side):
    """3x3-conv FLOPs of one decoded image (taming Decoder at latent side `side`)."""
    tot, res = 0, side
    mods = [("conv_in", dec.conv_in, res)]
    mods += [(n, m, res) for n, m in dec.mid.named_modules() if isinstance(m, torch.nn.Conv2d) and m.kernel_size == (3, 3)]
    for i_level in reversed(range(dec.num_resolutions)):
        up = dec.up[i_level]
        for blk in up.block:
            mods += [("c", blk.conv1, res), ("c", blk.conv2, res)]
        if i_level != 0:
            res *= 2
            mods.append(("u", up.upsample.conv, res))
    mods.append(("out", dec.conv_out, res))
    for _, m, r in mods:
        tot += 2 * r * r * m.in_channels * m.out_channels * 9
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    vae = VQGanVAE().to(dev).eval()
    codes = torch.randint(0, vae.num_tokens, (args.batch, 1024), device=dev)

    def run(torch_path):
        os.environ["DALLE_AMD_VQGAN_TORCH"] = "1" if torch_path else "0"
        out = vae.decode(codes)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.iters):
            out = vae.decode(codes)
        torch.cuda.synchronize()
        return out, (time.perf_counter() - t) / args.iters

    img, t_hip = run(False)
    ref, t_torch = run(True)
    fl = conv_flops(vae.decoder, 32) * args.batch
    print(json.dumps({"batch": args.batch, "hip_ms": round(t_hip * 1e3, 2), "torch_ms": round(t_torch * 1e3, 2),
                      "hip_images_per_s": round(args.batch / t_hip, 1), "torch_images_per_s": round(args.batch / t_torch, 1),
                      "hip_conv_tflops": round(fl / t_hip / 1e12, 1), "speedup": round(t_torch / t_hip, 2),
                      "max_abs_diff": round((img - ref).abs().max().item(), 4),
                      "mean_abs_diff": round((img - ref).abs().mean().item(), 5)}), flush=True)


if __name__ == "__main__":
    main()
