"""GradSync on gloo (2 ranks): grads handed over from inside backward (``notify``) give the same result
as a plain post-backward all-reduce, for the fp32 and the bf16 wire, under both algorithms; rs_ag shards
come from one preallocated buffer; ``tune_grad_sync`` returns the same selection on every rank."""
import pickle

import pytest
import torch
import torch.distributed as dist

from dalle_amd.optim import FlatArena
from dalle_amd.parallel.dp import GradSync, tune_grad_sync

from test_collab_cpu import _init, _run


def _params(rank):
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.zeros(n)) for n in (1000, 37, 4096, 513)]
    arena = FlatArena(ps)
    g = torch.Generator().manual_seed(10 + rank)
    for p in ps:
        p.grad.copy_(torch.randn(p.shape, generator=g))
    return ps, arena


def _worker(rank, world, port, q, dtype, algo):
    try:
        _init(rank, world, port)
        ps, arena = _params(rank)
        plain = GradSync(arena, world_size=world, grad_dtype=dtype, algo=algo, bucket_bytes=4096)
        saved = arena.grad.clone()
        plain.all_reduce()
        ref = arena.grad.clone()
        arena.grad.copy_(saved)
        gs = GradSync(arena, world_size=world, grad_dtype=dtype, algo=algo, bucket_bytes=4096)
        gs.notify([ps[2], ps[0]])          # final early, in the fused backward's hook order
        early = gs.early_elems
        gs.all_reduce()
        algo_sel, bucket, table = tune_grad_sync(arena, world, algos=("rccl", "rs_ag"), bucket_mb=(1, 2), reps=1)
        q.put(pickle.dumps((rank, torch.equal(arena.grad, ref), early, arena.grad.clone(), (algo_sel, bucket),
                            len(table), torch.equal(arena.grad, ref))))
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("algo", ["rccl", "rs_ag"])
def test_early_handover_matches_plain_allreduce(dtype, algo):
    (r0, same0, early0, g0, sel0, nt0, kept0), (r1, same1, early1, g1, sel1, nt1, _) = _run(_worker, 2, dtype, algo)
    assert same0 and same1                 # early hand-over == post-backward all-reduce, bitwise
    assert early0 > 0 and early1 == early0  # the bf16 wire is handed over early too
    assert torch.equal(g0, g1)             # replicas identical
    assert sel0 == sel1 and nt0 == 4       # tuner: same choice on every rank
    assert kept0                           # the tuner restores the arena grads


# ------------------------------------------------------------------------------------------------
# the real model over gloo: ranks bitwise identical and equal to one process on the concatenated batch
# (SURVEY §4 tier 6), for both all-reduce algorithms and both wire formats
def _train(world, batches, dtype="fp32", algo="rccl", steps=2):
    from dalle_amd.config import tiny
    from dalle_amd.models.dalle import DALLE
    from dalle_amd.optim import LAMB8bit

    torch.manual_seed(0)
    model = DALLE(tiny(False))
    arena = FlatArena(model.parameters())
    opt = LAMB8bit(model.parameters(), lr=0.01, max_grad_norm=4.0, reuse_grad_buffers=True, arena=arena)
    sync = GradSync(arena, world_size=world, bucket_bytes=256 * 1024, grad_dtype=dtype, algo=algo)  # several buckets
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


def _model_worker(rank, world, port, q, dtype, algo):
    try:
        _init(rank, world, port)
        full = _batches(7, 4)
        mine = [(t[2 * rank: 2 * rank + 2], im[2 * rank: 2 * rank + 2]) for t, im in full]
        q.put(pickle.dumps((rank, _train(world, mine, dtype, algo))))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
@pytest.mark.parametrize("algo", ["rccl", "rs_ag"])
def test_dp_ranks_identical_and_match_single_process(dtype, algo):
    (_, p0), (_, p1) = _run(_model_worker, 2, dtype, algo)
    assert torch.equal(p0, p1)  # bitwise identical replicas
    torch.set_num_threads(2)
    single = _train(1, _batches(7, 4))
    if dtype == "fp32":  # the averaged gradient differs from the single-process one by summation order only
        assert torch.allclose(p0, single, atol=2e-5, rtol=1e-4), (p0 - single).abs().max().item()
    else:  # bf16 wire: each rank's gradient rounded to bf16 -- the UPDATE agrees to a few percent of its norm
        init = _train(1, _batches(7, 4), steps=0)
        rel = ((p0 - single).norm() / (single - init).norm()).item()
        assert rel < 0.05, rel


def test_final_at_last_backward_use():
    from dalle_amd.ops.hip_ops import _final_at

    a, b, c, d = (torch.nn.Parameter(torch.zeros(1)) for _ in range(4))
    groups = [[a, b], [c, a], [b, d], [a, c]]   # shared params: final at their FIRST forward use
    out = _final_at(groups)
    ids = [[id(p) for p in g] for g in out]
    assert ids == [[id(a), id(b)], [id(c)], [id(d)], []]


# ------------------------------------------------------------------------------------------------
# world = 8 (the MI355X node): shard arithmetic b // N and the `% world` fallback (a bucket whose length is
# not a multiple of the world goes through a plain all_reduce and is scaled afterwards)
def _world8_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        torch.manual_seed(0)
        ps = [torch.nn.Parameter(torch.zeros(n)) for n in (1000, 37, 4096, 513, 77)]
        arena = FlatArena(ps, align=1)            # unpadded: odd range lengths
        out = {}
        for dtype in ("fp32", "bf16"):
            for algo in ("rccl", "rs_ag"):
                g = torch.Generator().manual_seed(10 + rank)
                arena.grad.copy_(torch.randn(arena.numel, generator=g))
                mine = arena.grad.clone()
                gs = GradSync(arena, world_size=world, grad_dtype=dtype, algo=algo, bucket_bytes=4 * 1001)
                gs.notify([ps[2], ps[0]])         # handed over early, out of order
                gs.all_reduce()
                allg = [torch.empty_like(mine) for _ in range(world)]
                dist.all_gather(allg, mine)
                ref = torch.stack(allg).double().mean(0)
                out[(dtype, algo)] = (arena.grad.clone(), float((arena.grad.double() - ref).abs().max()),
                                      len(gs.buckets), list(gs._fallback_ranges))
        q.put(pickle.dumps((rank, out)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_world8_shards_and_fallback_buckets():
    res = _run(_world8_worker, 8)
    for key in (("fp32", "rccl"), ("fp32", "rs_ag"), ("bf16", "rccl"), ("bf16", "rs_ag")):
        grads = [r[1][key][0] for r in res]
        assert all(torch.equal(grads[0], g) for g in grads[1:]), key      # every rank the same bits
        err = max(r[1][key][1] for r in res)
        assert err < (1e-5 if key[0] == "fp32" else 2e-2), (key, err)    # the average of the 8 ranks' grads
    # 5670 elements in 1001-element buckets: the rs_ag fallback ranges were exercised (1001 % 8 != 0)
    assert res[0][1][("fp32", "rs_ag")][2] == 6
