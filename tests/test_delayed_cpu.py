"""Delayed parameter update (``delay_optimizer_step=True``): the optimizer
steps on master copies concurrently with the next local step and the model sees the update one step
later. With a parameter-independent gradient the delayed trajectory must equal the synchronous one
exactly; the staleness window must be exactly one ``.step()`` call."""
import pickle

import pytest
import torch

from dalle_amd.optim import FlatArena, LAMB8bit, get_linear_schedule_with_warmup
from dalle_amd.parallel.optimizer import CollaborativeOptimizer

from test_collab_cpu import _init, _run


def _make(delay: bool, use_arena: bool, shape=(300, 500), seed=0, tracker_mode="auto"):
    torch.manual_seed(seed)
    w = torch.nn.Parameter(torch.randn(*shape) * 0.1)
    b = torch.nn.Parameter(torch.zeros(shape[0]))
    arena = FlatArena([w, b]) if use_arena else None
    groups = [{"params": [w], "weight_decay": 0.045}, {"params": [b], "weight_decay": 0.0}]
    opt = CollaborativeOptimizer(run_id="d", params=groups, arena=arena,
                                 optimizer=lambda ps: LAMB8bit(ps, lr=0.01, betas=(0.9, 0.96), eps=1e-6,
                                                               weight_decay=0.045, max_grad_norm=4.0),
                                 scheduler=lambda o: get_linear_schedule_with_warmup(o, 0, 20),
                                 target_batch_size=4, batch_size_per_step=2, reuse_grad_buffers=True,
                                 delay_optimizer_step=delay, offload_optimizer=True, tracker_mode=tracker_mode)
    return w, b, opt


def _const_grads(w, b, step):
    g = torch.Generator().manual_seed(100 + step)
    w.grad.add_(torch.randn(w.shape, generator=g))
    b.grad.add_(torch.randn(b.shape, generator=g))


@pytest.mark.parametrize("use_arena", [True, False])
def test_delayed_matches_synchronous(use_arena):
    ws, bs, sync = _make(False, use_arena)
    wd, bd, dly = _make(True, use_arena)
    assert dly.state_averager.runner is not None and sync.state_averager.runner is None
    for step in range(10):
        for w, b in ((ws, bs), (wd, bd)):
            if w.grad is None:
                w.grad, b.grad = torch.zeros_like(w), torch.zeros_like(b)
            _const_grads(w, b, step)
        before = wd.detach().clone()
        sync.step()
        dly.step()
        assert sync.local_epoch == dly.local_epoch
        if step % 2 == 1:  # this call completed an epoch: the delayed model is still one update behind
            assert dly.state_averager.pending
            assert torch.equal(wd.detach(), before)
            assert not torch.equal(ws.detach(), wd.detach())
        else:  # the boundary at the start of this call applied the previous epoch's update
            assert torch.equal(ws.detach(), wd.detach()) and torch.equal(bs.detach(), bd.detach())
    assert dly.apply_pending()
    assert torch.equal(ws.detach(), wd.detach()) and torch.equal(bs.detach(), bd.detach())
    # the optimizer state is the same too (positional state dicts)
    s1, s2 = sync.state_dict(), dly.state_dict()
    assert s1["state"]["local_epoch"] == s2["state"]["local_epoch"] == 5
    for k in s1["state"]:
        if k == "local_epoch":
            continue
        for name, v in s1["state"][k].items():
            if torch.is_tensor(v):
                assert torch.equal(v, s2["state"][k][name]), name
    assert [g["lr"] for g in sync.param_groups] == [g["lr"] for g in dly.param_groups]


def test_restore_drops_pending_update():
    w, b, opt = _make(True, True)
    snap_model = {"w": w.detach().clone(), "b": b.detach().clone()}
    snap_opt = opt.state_dict()
    for step in range(2):
        _const_grads(w, b, step)
        opt.step()
    assert opt.state_averager.pending
    # a backup restore while the update is in flight: the model keeps the restored values
    w.data.copy_(snap_model["w"])
    opt.load_state_dict(snap_opt)
    assert not opt.apply_pending()
    assert torch.equal(w.detach(), snap_model["w"])
    # and the next epoch steps from the restored values
    for step in range(2):
        _const_grads(w, b, step)
        opt.step()
    opt.apply_pending()
    assert not torch.equal(w.detach(), snap_model["w"]) and torch.isfinite(w).all()


def _delayed_dp_worker(rank, world, port, q, delay):
    try:
        _init(rank, world, port)
        # homogeneous peers, one global step per local step: the static tracker (deterministic epochs)
        w, b, opt = _make(delay, True, shape=(64, 96), seed=0, tracker_mode="static")
        for step in range(6):
            _const_grads(w, b, 10 * rank + step)
            opt.step()
        opt.apply_pending()
        q.put(pickle.dumps((rank, opt.local_epoch, w.detach().clone(), b.detach().clone())))
        torch.distributed.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_delayed_two_peers_match_synchronous():
    sync = _run(_delayed_dp_worker, 2, False)
    dly = _run(_delayed_dp_worker, 2, True)
    # target 4 samples, 2 peers x 2 samples per step -> an epoch every step
    assert [r[1] for r in sync] == [r[1] for r in dly] == [6, 6]
    for (_, _, ws, bs), (_, _, wd, bd) in zip(sync, dly):
        assert torch.equal(ws, wd) and torch.equal(bs, bd)
    assert torch.equal(dly[0][2], dly[1][2])
