"""Data-parallel step (bench.py's path) on gloo: bucketed all-reduce over the flat gradient arena
keeps ranks bitwise identical and equals one process on the concatenated batch (SURVEY §4 tier 6)."""
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


def _train(world, rank, batches, steps=2):
    from dalle_amd.config import tiny
    from dalle_amd.models.dalle import DALLE
    from dalle_amd.optim import FlatArena, LAMB8bit
    from dalle_amd.parallel.dp import GradSync

    torch.manual_seed(0)
    cfg = tiny(False)
    model = DALLE(cfg)
    arena = FlatArena(model.parameters())
    opt = LAMB8bit(model.parameters(), lr=0.01, max_grad_norm=4.0, reuse_grad_buffers=True, arena=arena)
    sync = GradSync(arena, world_size=world, bucket_bytes=256 * 1024)  # several buckets
    for i in range(steps):
        text, image = batches[i]
        arena.zero_grad()
        model(text, image, return_loss=True).backward()
        sync.all_reduce()
        opt.step()
    return arena.data.clone()


def _batches(seed, n):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randint(1, 900, (n, 64), generator=g), torch.randint(0, 512, (n, 256), generator=g)) for _ in range(2)]


def _worker(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
        torch.set_num_threads(2)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        full = _batches(7, 4)
        mine = [(t[2 * rank: 2 * rank + 2], im[2 * rank: 2 * rank + 2]) for t, im in full]
        q.put(pickle.dumps((rank, _train(world, rank, mine))))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_dp_ranks_identical_and_match_single_process():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([pickle.loads(q.get()) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
    assert res[0][0] != "error", res[0][2]
    assert res[1][0] != "error", res[1][2]
    assert torch.equal(res[0][1], res[1][1])  # bitwise identical replicas
    torch.set_num_threads(2)
    single = _train(1, 0, _batches(7, 4))
    assert torch.allclose(res[0][1], single, atol=2e-5, rtol=1e-4)


def _worker_early(rank, world, port, q):
    """GradSync.notify (the hand-off the fused backward makes) on a subset of parameters before
    all_reduce: same averaged gradient, bitwise, as one all_reduce of the whole arena."""
    try:
        os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
        torch.set_num_threads(2)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dalle_amd.optim import FlatArena
        from dalle_amd.parallel.dp import GradSync

        torch.manual_seed(0)
        ps = [torch.nn.Parameter(torch.zeros(s)) for s in [(300, 40), (7,), (5000,), (64, 64), (3,)]]
        arena = FlatArena(ps)
        outs = []
        for early in (False, True):
            g = torch.Generator().manual_seed(100 + rank)
            arena.grad.copy_(torch.randn(arena.numel, generator=g))
            sync = GradSync(arena, world_size=world, bucket_bytes=4096 * 4)
            if early:
                sync.notify([ps[2], ps[0]])   # two non-adjacent tensors, out of order
                sync.notify([ps[3]])
            sync.all_reduce()
            outs.append((arena.grad.clone(), sync.last_early_elems))
        q.put(pickle.dumps((rank, outs)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_grad_sync_early_handoff_equals_single_all_reduce():
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_worker_early, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([pickle.loads(q.get()) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(60)
    for r in res:
        assert r[0] != "error", r[2]
    (plain0, n0), (early0, n1) = res[0][1]
    assert n0 == 0 and n1 > 0
    assert torch.equal(plain0, early0)
    assert torch.equal(res[0][1][1][0], res[1][1][1][0])


def test_final_at_last_backward_use():
    from dalle_amd.ops.hip_ops import _final_at

    a, b, c, d = (torch.nn.Parameter(torch.zeros(1)) for _ in range(4))
    groups = [[a, b], [c, a], [b, d], [a, c]]   # shared params: final at their FIRST forward use
    out = _final_at(groups)
    ids = [[id(p) for p in g] for g in out]
    assert ids == [[id(a), id(b)], [id(c)], [id(d)], []]
