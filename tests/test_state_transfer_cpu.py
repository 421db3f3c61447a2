"""``load_state_from_peers`` (reference callback.py:41, run_aux_peer.py:48) moves the optimizer
state as tensors on the group, not through pickle: only the skeleton (hyper-parameters, step counters,
tensor shapes / dtypes) is an object broadcast. Checked on CPU/gloo with 2 ranks and an 8-bit LAMB whose
moments are several MB: no pickled payload over 1 MB, and the joiner's state equals the donor's."""
import pickle

import pytest
import torch
import torch.distributed as dist

from test_collab_cpu import _init, _run


def _worker(rank, world, port, q, chunk=None):
    try:
        _init(rank, world, port)
        from dalle_amd.optim import LAMB8bit, get_linear_schedule_with_warmup
        from dalle_amd.parallel import optimizer as copt_mod
        from dalle_amd.parallel.optimizer import CollaborativeOptimizer

        if chunk:
            copt_mod.STATE_CHUNK_BYTES = chunk   # windows that cut through tensors

        sizes = []
        orig = dist.broadcast_object_list

        def spy(objs, *a, **kw):
            sizes.append(len(pickle.dumps(objs)))
            return orig(objs, *a, **kw)

        dist.broadcast_object_list = spy
        torch.manual_seed(rank)  # different init on purpose
        w = torch.nn.Parameter(torch.randn(2048, 1536))
        b = torch.nn.Parameter(torch.randn(1536))
        opt = CollaborativeOptimizer(run_id="st", params=[w, b], optimizer=lambda ps: LAMB8bit(ps, lr=0.01),
                                     scheduler=lambda o: get_linear_schedule_with_warmup(o, 10, 100),
                                     target_batch_size=4, batch_size_per_step=2, reuse_grad_buffers=True)
        if rank == 0:
            opt.local_epoch = 5
            for _ in range(3):
                w.grad, b.grad = torch.randn_like(w), torch.randn_like(b)
                opt.opt.step()
                opt.scheduler.step()
        received = opt.load_state_from_peers()
        st = opt.opt.state[w]
        out = (rank, received, opt.local_epoch, w.detach().clone(), st["state1"].clone(), st["state2"].clone(),
               st["absmax1"].clone(), opt.opt.state[b]["state1"].clone(), st["step"], opt.scheduler.state_dict()["last_epoch"],
               max(sizes))
        dist.broadcast_object_list = orig
        q.put(pickle.dumps(out))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


@pytest.mark.parametrize("chunk", [None, 1000003])
def test_state_transfer_moves_tensors_not_pickles(chunk):
    """(chunk: the transfer's staging window -- the default 128 MB, or ~1 MB so every moment tensor straddles
    several windows)"""
    (r0, rec0, ep0, w0, s10, s20, a0, sb0, step0, le0, big0), (r1, rec1, ep1, w1, s11, s21, a1, sb1, step1, le1, big1) = \
        _run(_worker, 2, chunk)
    assert not rec0 and rec1 and ep0 == ep1 == 5
    assert torch.equal(w0, w1)
    assert s10.dtype == torch.uint8 and s10.numel() > 1 << 20
    assert torch.equal(s10, s11) and torch.equal(s20, s21) and torch.equal(a0, a1) and torch.equal(sb0, sb1)
    assert step0 == step1 == 3 and le0 == le1 == 3
    assert max(big0, big1) < 1 << 20, (big0, big1)  # the 3 MB of moments did not go through pickle
