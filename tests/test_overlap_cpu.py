"""Backward-overlapped gradient rounds (``GradientAverager.arm`` -> ``GradSync``) on CPU/gloo, with the
fused backward's grad-ready hook driven by hand (on the GPU the fused stacks call it per layer):

* with a collaborative grad scaler, the round's in-flight all-reduce completes BEFORE the unscale and
  the overflow check (they used to run on the compute stream while RCCL still reduced the same memory);
  with a power-of-two scale the result is bitwise the one of the non-overlapped round;
* a second hooked backward before ``step()`` raises instead of all-reducing the same range twice, and a
  trainer with gradient accumulation disarms the overlap altogether."""
import pickle

import pytest
import torch

from dalle_amd.optim import FlatArena
from dalle_amd.optim.grad_scaler import CollaborativeGradScaler
from dalle_amd.parallel.optimizer import CollaborativeOptimizer

from test_collab_cpu import _init, _run


def _make(overlap: bool, rank: int):
    torch.manual_seed(0)
    w = torch.nn.Parameter(torch.randn(64, 96) * 0.1)
    b = torch.nn.Parameter(torch.zeros(64))
    arena = FlatArena([w, b])
    opt = CollaborativeOptimizer(run_id="ov", params=[w, b], arena=arena,
                                 optimizer=lambda ps: torch.optim.SGD(ps, lr=0.5),
                                 target_batch_size=8, batch_size_per_step=2, reuse_grad_buffers=True,
                                 tracker_mode="static", overlap_grad_averaging=overlap, recovery="detach",
                                 average_state_every=0)
    return w, b, opt


def _backward(w, b, rank, step, scale, hook=True):
    """What the fused backward does: scaled grads land in the arena, then the hook hands them over."""
    from dalle_amd.ops import hip_ops

    g = torch.Generator().manual_seed(1000 * rank + step)
    w.grad.add_(torch.randn(w.shape, generator=g) * scale)
    b.grad.add_(torch.randn(b.shape, generator=g) * scale)
    if hook and hip_ops._grad_ready_hook is not None:
        hip_ops._grad_ready_hook([w, b])


def _scaler_worker(rank, world, port, q, overlap):
    try:
        _init(rank, world, port)
        w, b, opt = _make(overlap, rank)
        scaler = CollaborativeGradScaler(init_scale=2.0 ** 10)
        rounds = []
        for step in range(8):
            if w.grad is None:
                w.grad, b.grad = torch.zeros_like(w), torch.zeros_like(b)
            rounds.append(opt.grad_averager._armed)
            _backward(w, b, rank, step, scaler.get_scale())
            scaler.step(opt)
            scaler.update()
        q.put(pickle.dumps((rank, w.detach().clone(), b.detach().clone(), rounds, opt.grad_averager.overlapped_rounds)))
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_scaled_overlapped_round_matches_plain_round():
    on = _run(_scaler_worker, 2, True)
    off = _run(_scaler_worker, 2, False)
    (_, w0, b0, armed0, n0), (_, w1, b1, _, _) = on
    (_, w0f, b0f, armed_f, nf), _ = off
    assert n0 == 4 and nf == 0 and any(armed0) and not any(armed_f)  # 8 steps x 2 peers x 2 samples, 8 per round
    assert torch.equal(w0, w1) and torch.equal(b0, b1)               # replicas identical
    assert torch.equal(w0, w0f) and torch.equal(b0, b0f)             # 2^-10 unscale is exact either order


def _double_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        w, b, opt = _make(True, rank)
        w.grad, b.grad = torch.zeros_like(w), torch.zeros_like(b)
        out = {}
        # a round closes every 2nd step (2 peers x 2 samples, target 8)
        for step in range(3):
            _backward(w, b, rank, step, 1.0)
            opt.step()
        assert opt.grad_averager._armed
        _backward(w, b, rank, 3, 1.0)
        try:
            _backward(w, b, rank, 4, 1.0)  # an extra hooked backward before step()
            out["raised"] = False
        except RuntimeError as e:
            out["raised"] = "handed over twice" in str(e)
        opt.grad_averager.abandon_overlap()
        opt.grad_averager.reset_accumulated_grads_()
        # a trainer with gradient accumulation declares its backwards per step: no overlap at all
        opt.set_backwards_per_step(4)
        out["armed_after_accum"] = opt.grad_averager._armed
        for step in range(8):
            _backward(w, b, rank, 10 + step, 1.0)
            out.setdefault("armed_any", False)
            out["armed_any"] |= opt.grad_averager._armed
            opt.step()
        q.put(pickle.dumps((rank, out)))
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_second_hooked_backward_raises_and_accumulation_disarms():
    for rank, out in _run(_double_worker, 2):
        assert out["raised"], out
        assert not out["armed_after_accum"] and not out["armed_any"], out


def test_trainer_declares_its_accumulation():
    from dalle_amd.train.trainer import CollaborativeHFTrainer
    import inspect

    src = inspect.getsource(CollaborativeHFTrainer.train)
    assert "set_backwards_per_step" in src


def _failed_round_worker(rank, world, port, q):
    """An armed, scaled round whose overlapped all-reduce failed (dead / slow peer): the overflow check must
    run locally -- a group all-reduce queued behind the broken collective would hang instead of falling back."""
    try:
        _init(rank, world, port)
        w, b, opt = _make(True, rank)
        scaler = CollaborativeGradScaler(init_scale=2.0 ** 10)
        seen = []
        real_check = scaler.unscale_and_check

        def check(*a, **kw):
            seen.append(kw.get("local_only", False))
            return real_check(*a, **kw)

        scaler.unscale_and_check = check
        ga = opt.grad_averager

        def failed_round(epoch, batch_size):
            ga.abandon_overlap()          # the in-flight round died: no collective completes
            ga.comm_failed = True
            return False

        ga._step_overlapped = failed_round
        w.grad, b.grad = torch.zeros_like(w), torch.zeros_like(b)
        armed = []
        for step in range(4):
            armed.append(ga._armed)
            _backward(w, b, rank, step, scaler.get_scale())
            scaler.step(opt)
            scaler.update()
        q.put(pickle.dumps((rank, seen, armed, bool(torch.isfinite(w).all()))))
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_failed_armed_scaled_round_checks_overflow_locally():
    for rank, seen, armed, finite in _run(_failed_round_worker, 2):
        assert any(armed), armed          # the round that failed was an overlapped one
        assert seen and seen[0] is True, seen
        assert finite
