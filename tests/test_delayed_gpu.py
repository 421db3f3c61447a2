"""Delayed parameter update on MI355X: the fused 8-bit LAMB runs on a side HIP stream over the
master arena while the main stream keeps computing on the stale model parameters (event-ordered,
``dalle_amd/parallel/delayed.py``). Must equal the synchronous fused path bitwise."""
import pytest
import torch

from dalle_amd.optim import FlatArena, LAMB8bit, get_linear_schedule_with_warmup
from dalle_amd.parallel.optimizer import CollaborativeOptimizer

pytestmark = pytest.mark.gpu


def _make(delay, dev, offload_device=None):
    torch.manual_seed(0)
    w = torch.nn.Parameter(0.05 * torch.randn(1024, 3072, device=dev))
    b = torch.nn.Parameter(torch.zeros(1024, device=dev))
    s = torch.nn.Parameter(torch.full((1024,), 0.1, device=dev))
    arena = FlatArena([w, b, s], device=dev)
    groups = [{"params": [w, s], "weight_decay": 0.045}, {"params": [b], "weight_decay": 0.0}]
    opt = CollaborativeOptimizer(run_id="dg", params=groups, arena=arena,
                                 optimizer=lambda ps: LAMB8bit(ps, lr=0.0025, betas=(0.9, 0.96), eps=1e-6,
                                                               weight_decay=0.045, max_grad_norm=4.0,
                                                               clamp_value=10000.0, reuse_grad_buffers=True),
                                 scheduler=lambda o: get_linear_schedule_with_warmup(o, 0, 50),
                                 target_batch_size=4, batch_size_per_step=2, reuse_grad_buffers=True,
                                 delay_optimizer_step=delay, offload_optimizer=True, offload_device=offload_device)
    return (w, b, s), arena, opt


def test_delayed_side_stream_matches_sync(cuda):
    ps_sync, ar_sync, sync = _make(False, cuda)
    ps_dly, ar_dly, dly = _make(True, cuda)
    assert dly.state_averager.runner.cuda
    x = torch.randn(4096, 1024, device=cuda)
    for step in range(8):
        g = torch.Generator(device=cuda).manual_seed(7 + step)
        noise = torch.randn(ar_sync.numel, device=cuda, generator=g)
        ar_sync.grad.add_(noise)
        ar_dly.grad.add_(noise)
        sync.step()
        before = ar_dly.data.clone()
        dly.step()
        # main-stream work queued behind the side-stream launch sees the stale parameters
        y = x @ ps_dly[0]
        assert torch.isfinite(y).all()
        if step % 2 == 1:  # this call launched the update: the model is one update behind
            assert torch.equal(ar_dly.data, before) and not torch.equal(ar_sync.data, ar_dly.data)
        else:  # the boundary at the start of this call applied it
            assert torch.equal(ar_sync.data, ar_dly.data)
    dly.apply_pending()
    torch.cuda.synchronize()
    assert torch.equal(ar_sync.data, ar_dly.data)
    assert sync.local_epoch == dly.local_epoch == 4


@pytest.mark.parametrize("delay", [False, True])
def test_host_offload_matches_hbm_optimizer(cuda, delay):
    """offload_device="cpu": pinned host master + CPU LAMB step (thread when delayed) == the HBM fused
    path up to fp32 rounding of the two LAMB implementations (8-bit moments: same block maps)."""
    ps_ref, ar_ref, ref = _make(False, cuda)
    ps_off, ar_off, off = _make(delay, cuda, offload_device="cpu")
    assert off._master.offloaded and off._master.arena.data.is_pinned()
    assert not off.state_averager.optimizer._get_fused()  # the CPU path
    for step in range(8):
        g = torch.Generator(device=cuda).manual_seed(7 + step)
        noise = torch.randn(ar_ref.numel, device=cuda, generator=g)
        ar_ref.grad.add_(noise)
        ar_off.grad.add_(noise)
        ref.step()
        off.step()
    off.apply_pending()
    torch.cuda.synchronize()
    rel = ((ar_ref.data - ar_off.data).norm() / ar_ref.data.norm()).item()
    assert rel < 1e-4, rel
    assert off.local_epoch == 4


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_generic_host_offload_optimizer_on_hbm_params(cuda, dtype):
    """HostOffloadOptimizer: any torch optimizer (Adam here) on pinned host copies of HBM parameters ==
    the same optimizer stepping on the device (fp32: to rounding; bf16 params: fp32 host master per step)."""
    import sys, os
    sys.path.insert(0, os.path.dirname(__file__))
    from test_optim_cpu import _offload_vs_plain

    a, b, off = _offload_vs_plain(cuda, dtype)
    torch.cuda.synchronize()
    assert off._host.is_pinned() and all(v["exp_avg"].device.type == "cpu" for v in off.inner.state.values())
    for x, y in zip(a, b):
        assert y.device.type == "cuda" and y.dtype == dtype
        tol = dict(rtol=1e-5, atol=1e-6) if dtype == torch.float32 else dict(rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(x.float(), y.float(), **tol)
