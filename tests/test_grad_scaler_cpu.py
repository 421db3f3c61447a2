"""Collaborative (global-step deferred) loss scaler, SURVEY D28: unscale + overflow check happen once per
global step across all peers; local steps never change the scale."""
import os
import pickle
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, overflow_rank):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        torch.set_num_threads(1)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dalle_amd.optim.grad_scaler import CollaborativeGradScaler
        from dalle_amd.parallel.optimizer import CollaborativeOptimizer

        p = torch.nn.Parameter(torch.zeros(64))
        opt = CollaborativeOptimizer(run_id="gs", params=[p], optimizer=lambda ps: torch.optim.SGD(ps, lr=1.0),
                                     target_batch_size=8, batch_size_per_step=2, reuse_grad_buffers=True,
                                     average_state_every=0, tracker_mode="static")  # homogeneous: deterministic epochs
        scaler = CollaborativeGradScaler(init_scale=1024.0, growth_interval=1)
        scales, steps = [], 0
        while opt.local_epoch == 0:
            g = torch.full_like(p, float(rank + 1))
            if rank == overflow_rank and steps == 0:
                g[3] = float("inf")
            scaled = g * scaler.get_scale()  # == grad of scaler.scale(loss)
            p.grad = scaled.clone() if p.grad is None else p.grad.add_(scaled)
            scaler.step(opt)
            scaler.update()
            scales.append(scaler.get_scale())
            steps += 1
        q.put(pickle.dumps((rank, steps, p.detach().clone(), scales)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def _run(overflow_rank):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, overflow_rank)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = [pickle.loads(q.get()) for _ in range(2)]
    for pr in procs:
        pr.join(60)
    for r in res:
        assert r[0] != "error", r[2]
    return sorted(res, key=lambda r: r[0])


def test_scaled_global_step_matches_unscaled():
    (r0, steps, p0, scales0), (_, _, p1, _) = _run(overflow_rank=-1)
    assert steps == 2  # 2 peers x 2 samples per step -> 8 samples after 2 local steps
    # per-peer mean grads 1 and 2 weighted equally -> averaged grad 1.5, SGD lr 1 from zero
    assert torch.allclose(p0, torch.full_like(p0, -1.5), atol=1e-5)
    assert torch.allclose(p0, p1)
    assert scales0[0] == 1024.0  # a local-only step leaves the scale alone
    assert scales0[-1] == 2048.0  # clean global step with growth_interval=1 grows it


def test_overflow_on_one_peer_skips_the_update_everywhere():
    (_, steps, p0, scales0), (_, _, p1, scales1) = _run(overflow_rank=1)
    assert torch.equal(p0, torch.zeros_like(p0)) and torch.equal(p1, torch.zeros_like(p1))
    assert scales0[-1] == 512.0 and scales1[-1] == 512.0  # both peers backed off
