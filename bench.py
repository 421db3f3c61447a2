#!/usr/bin/env python3
"""Headline benchmark: training samples/s (whole node) of DALL-E d_model=1024, 24 layers,
256 text + 32x32 image tokens, bf16 data-parallel on 1/2/4/8 MI355X (BASELINE.json config 2).

One process per GPU (torchrun), RCCL over xGMI. Every timed step is a full training step:
forward + backward (fused HIP kernels), gradient all-reduce across ranks (bucketed, RCCL),
global grad-norm clip and a LAMB optimizer update on every parameter -- i.e. the collaborative
optimizer with ``target_batch_size`` equal to the global batch, so each step is a global step.

Data: synthetic LAION-shaped pairs (256 caption ids padded with 1, 1024 VQGAN codes), random-init
weights. ``python bench.py --gpus N --steps K --warmup W``; rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from dalle_amd.config import get_config  # noqa: E402
from dalle_amd.data.synthetic import synthetic_batch  # noqa: E402
from dalle_amd.models.dalle import DALLE  # noqa: E402
from dalle_amd.optim import FlatArena, LAMB8bit  # noqa: E402
from dalle_amd.parallel.dp import GradSync  # noqa: E402

MODEL_NAMES = {
    "bench24": "DALL-E d_model=1024, 24 layers, 256 text + 32x32 image tokens",
    "dalle-1024-24l": "DALL-E d_model=1024, 24 layers, 256 text + 32x32 image tokens",
    "reference": "DALL-E d_model=1024, 64 layers (5 shared blocks), reversible, 256 text + 32x32 image tokens",
    "dalle-1.3b": "DALL-E ~1.3B, reversible, 256 text + 32x32 image tokens",
}
BASELINE_VALUE = None  # the reference publishes no throughput numbers


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("BENCH_BATCH", 48)), help="per-GPU micro-batch (48: best measured, 74 GB of 288)")
    ap.add_argument("--model", default="bench24")
    ap.add_argument("--optim-bits", type=int, default=32, choices=[8, 32])
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--compression", default="none", choices=["none", "powersgd", "uniform8bit"],
                    help="gradient averaging: plain bucketed all-reduce, PowerSGD rank-4 with error feedback "
                         "(BASELINE config 3) or the hivemind size-adaptive fp16 / uniform-8-bit butterfly")
    ap.add_argument("--powersgd-rank", type=int, default=4)
    ap.add_argument("--profile-steps", type=int, default=0,
                    help="after the timed run: K more steps with per-phase timing (+ torch.profiler trace)")
    ap.add_argument("--trace", default="", help="chrome trace path for the --profile-steps pass")
    ap.add_argument("--no-recompute", action="store_true",
                    help="reversible presets: keep the activations instead of rebuilding them in backward")
    ap.add_argument("--tunable", default="off", choices=["auto", "use", "tune", "off"],
                    help="hipBLASLt solution selection for the library GEMMs (dalle_amd/utils/tuning.py)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; more ranks than GPUs (a rehearsal of the multi-rank path on a 1-GPU box, with
    # BENCH_BACKEND=gloo) share devices round-robin
    dev_index = local_rank % max(1, torch.cuda.device_count())
    backend = os.environ.get("BENCH_BACKEND", "nccl")
    if world > 1:
        torch.cuda.set_device(dev_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", dev_index)
    torch.backends.cuda.matmul.allow_tf32 = False
    from dalle_amd.utils.tuning import setup_gemm_tuning
    tuning = setup_gemm_tuning(args.tunable if (args.tunable != "tune" or rank == 0) else "use")

    cfg = get_config(args.model)
    if args.no_recompute:
        cfg.reversible_recompute = False
    torch.manual_seed(1234)
    model = DALLE(cfg).to(device)
    arena = FlatArena(model.parameters(), device=device)
    if world > 1:  # identical init on every rank
        dist.broadcast(arena.data, 0)
    no_decay = ["bias", "LayerNorm.weight"]  # task.py:138-150 (only biases match dalle-pytorch names)
    named = list(model.named_parameters())
    groups = [
        {"params": [p for n, p in named if not any(nd in n for nd in no_decay)], "weight_decay": 0.045},
        {"params": [p for n, p in named if any(nd in n for nd in no_decay)], "weight_decay": 0.0},
    ]
    opt = LAMB8bit(groups, lr=0.0025, betas=(0.9, 0.96), eps=1e-6, weight_decay=0.045, clamp_value=10000.0,
                   max_grad_norm=4.0, reuse_grad_buffers=True, optim_bits=args.optim_bits, arena=arena)
    sync = GradSync(arena, world_size=world, grad_dtype=args.grad_dtype)
    if args.compression == "powersgd":
        # compression work runs at every world size (the all-reduces are skipped only when world == 1)
        from dalle_amd.parallel.powersgd import PowerSGD
        psgd = PowerSGD([p for _, p in named], rank=args.powersgd_rank, seed=0)
        reduce_grads = psgd.allreduce_
    elif args.compression == "uniform8bit":
        from dalle_amd.parallel.averaging import allreduce_weighted
        from dalle_amd.parallel.compression import reference_averaging_compression
        comp = reference_averaging_compression()

        def reduce_grads():
            allreduce_weighted(arena.grad, 1.0, compression=comp)  # a no-op on one GPU
    else:
        reduce_grads = sync.all_reduce

    gen = torch.Generator().manual_seed(1000 + rank)
    batches = [synthetic_batch(args.batch, cfg.text_seq_len, cfg.image_seq_len, cfg.num_text_tokens,
                               cfg.num_image_tokens, gen, device=device) for _ in range(4)]

    from dalle_amd.utils.profiling import StepTimer, prof_range

    def step(i, timer=None):
        phase = timer if timer is not None else (lambda name: prof_range(name))
        b = batches[i % len(batches)]
        arena.zero_grad()
        with phase("forward"):
            loss = model(b["input_ids"], b["image"], mask=b["attention_mask"], return_loss=True)
        with phase("backward"):
            loss.backward()
        with phase("grad_allreduce"):
            reduce_grads()
        with phase("optimizer"):
            opt.step()
        return loss

    for i in range(args.warmup):
        loss = step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    final_loss = float(loss.item())

    samples = args.batch * world * args.steps
    value = samples / elapsed
    ms = elapsed / args.steps * 1000
    if rank == 0:
        tflops = cfg.train_flops_per_sample() * value / world / 1e12  # model FLOPs (no recompute)
        hw_tflops = cfg.train_flops_per_sample(include_recompute=True) * value / world / 1e12
        print(json.dumps({
            "metric": "training samples/sec (whole node), DALL-E d_model=1024 at 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_VALUE is None else value / BASELINE_VALUE,
            "dtype": "bf16",
            "data": "synthetic LAION-shaped pairs (256 caption ids + 32x32 VQGAN codes), random-init weights",
            "config": {"model": MODEL_NAMES.get(args.model, args.model),
                       "preset": args.model, "global_batch": args.batch * world, "per_gpu_batch": args.batch,
                       "seq_len": cfg.seq_len, "parallelism": f"dp{world}",
                       "optimizer": f"LAMB ({args.optim_bits}-bit moments) + global clip 4.0",
                       "grad_allreduce_dtype": args.grad_dtype, "gemm_selection": tuning,
                       "reversible": ("recompute" if cfg.reversible_recompute else "stored activations") if cfg.reversible else "no",
                       "grad_compression": args.compression if args.compression != "powersgd"
                       else f"powersgd-rank{args.powersgd_rank}"},
            "model_tflops_per_gpu": round(tflops, 1),
            "hw_tflops_per_gpu": round(hw_tflops, 1),
            "max_mem_gb": round(torch.cuda.max_memory_allocated(device) / 2 ** 30, 1),
            "loss": round(final_loss, 4),
        }), flush=True)
    if args.profile_steps:
        # untimed diagnostic pass: per-phase wall times (synchronised) and an optional trace
        timer = StepTimer()
        prof = None
        if args.trace:
            prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                      torch.profiler.ProfilerActivity.CUDA])
            prof.__enter__()
        for i in range(args.profile_steps):
            step(i, timer)
        if prof is not None:
            prof.__exit__(None, None, None)
            if rank == 0:
                prof.export_chrome_trace(args.trace)
        if rank == 0:
            print("# phase ms/step: " + json.dumps(timer.summary()), file=sys.stderr, flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
