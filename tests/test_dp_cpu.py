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
