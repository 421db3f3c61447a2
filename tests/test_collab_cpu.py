"""Collaboration plumbing on CPU/gloo with local peer processes (SURVEY §4 tiers 4-5)."""
import os
import pickle
import socket
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dalle_amd.parallel.compression import Float16Compression, SizeAdaptiveCompression, Uniform8BitQuantization, reference_averaging_compression
from dalle_amd.parallel.averaging import shard_bounds


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _run(fn, world, *args):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    results = [pickle.loads(q.get()) for _ in range(world)]
    for p in procs:
        p.join(60)
    for r in results:
        if isinstance(r, BaseException) or (isinstance(r, tuple) and r and r[0] == "error"):
            raise AssertionError(r)
    return sorted(results, key=lambda r: r[0])


# ------------------------------------------------------------------------------------------------
def _weighted_avg_worker(rank, world, port, q, mode):
    try:
        _init(rank, world, port)
        from dalle_amd.parallel.optimizer import CollaborativeOptimizer
        from dalle_amd.optim import LAMB8bit

        torch.manual_seed(0)
        p = torch.nn.Parameter(torch.zeros(200, 300))
        bs = [3, 5][rank]  # heterogeneous peers
        comp = {"none": None, "fp16": Float16Compression(), "8bit": reference_averaging_compression()}[mode]
        opt = CollaborativeOptimizer(run_id="t", params=[p], optimizer=lambda ps: torch.optim.SGD(ps, lr=1.0),
                                     target_batch_size=16, batch_size_per_step=bs, reuse_grad_buffers=True,
                                     grad_compression=comp, average_state_every=0)
        grads_seen = []
        steps = 0
        while opt.local_epoch == 0:
            g = torch.full_like(p, float(rank + 1)) + 0.01 * steps
            grads_seen.append(g)
            p.grad = g.clone() if p.grad is None else p.grad.add_(g)
            opt.step()
            steps += 1
        q.put(pickle.dumps((rank, steps, p.detach().clone(), sum(grads_seen) / len(grads_seen), bs * steps)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


@pytest.mark.parametrize("mode", ["none", "fp16", "8bit"])
def test_sample_weighted_averaging_and_epoch_trigger(mode):
    res = _run(_weighted_avg_worker, 2, mode)
    (r0, steps0, p0, mean0, s0), (r1, steps1, p1, mean1, s1) = res
    assert steps0 == steps1  # collective progress: same step ends the epoch on both peers
    assert s0 + s1 >= 16 and (s0 - 3) + (s1 - 5) < 16
    expected = -(s0 * mean0 + s1 * mean1) / (s0 + s1)  # SGD lr=1 from zero
    tol = {"none": 1e-6, "fp16": 2e-3, "8bit": 5e-2}[mode]
    assert torch.allclose(p0, expected, atol=tol * expected.abs().max().item())
    assert torch.allclose(p0, p1, atol=tol * expected.abs().max().item())


# ------------------------------------------------------------------------------------------------
def _powersgd_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from dalle_amd.parallel.powersgd import PowerSGD

        torch.manual_seed(1)
        A = torch.randn(64, 4) @ torch.randn(4, 48)  # rank-4 gradient (same on all peers)
        p = torch.nn.Parameter(torch.zeros(64, 48))
        b = torch.nn.Parameter(torch.zeros(48))
        psgd = PowerSGD([p, b], rank=4)
        errs = []
        for it in range(3):
            p.grad = A * (rank + 1)
            b.grad = torch.full((48,), float(rank))
            psgd.allreduce_()
            errs.append(((p.grad - A * 1.5).norm() / (A * 1.5).norm()).item())
        q.put(pickle.dumps((rank, errs, b.grad.clone(), psgd.compression_ratio())))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_powersgd_exact_on_low_rank_gradients():
    res = _run(_powersgd_worker, 2)
    for rank, errs, bgrad, ratio in res:
        assert errs[-1] < 1e-4, errs
        assert torch.allclose(bgrad, torch.full((48,), 0.5))
        assert ratio > 1.0


# ------------------------------------------------------------------------------------------------
def _late_joiner_worker(rank, world, port, q):
    try:
        _init(rank, world, port)
        from dalle_amd.parallel.optimizer import CollaborativeOptimizer
        from dalle_amd.optim import LAMB8bit, get_linear_schedule_with_warmup

        torch.manual_seed(rank)  # different init on purpose
        p = torch.nn.Parameter(torch.randn(100, 700))
        opt = CollaborativeOptimizer(run_id="t", params=[p], optimizer=lambda ps: LAMB8bit(ps, lr=0.01),
                                     scheduler=lambda o: get_linear_schedule_with_warmup(o, 10, 100),
                                     target_batch_size=4, batch_size_per_step=2, reuse_grad_buffers=True)
        if rank == 0:
            opt.local_epoch = 7
            p.grad = torch.randn_like(p)
            opt.opt.step()  # create optimizer state on the donor
        opt.load_state_from_peers()
        st = opt.opt.state[p]
        q.put(pickle.dumps((rank, opt.local_epoch, p.detach().clone(), st["state1"].clone(), st["absmax1"].clone())))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_load_state_from_peers():
    (r0, e0, p0, s0, a0), (r1, e1, p1, s1, a1) = _run(_late_joiner_worker, 2)
    assert e0 == e1 == 7
    assert torch.equal(p0, p1) and torch.equal(s0, s1) and torch.equal(a0, a1)
    assert s1.dtype == torch.uint8


# ------------------------------------------------------------------------------------------------
def test_compression_roundtrips():
    torch.manual_seed(0)
    x = torch.randn(100000)
    assert torch.allclose(Float16Compression().roundtrip(x), x, rtol=1e-3, atol=1e-4)
    u = Uniform8BitQuantization()
    c = u.compress(x)
    assert c["idx"].dtype == torch.uint8 and c["codebook"].shape == (256,)
    y = u.roundtrip(x)
    assert ((y - x).norm() / x.norm()).item() < 0.05
    sa = reference_averaging_compression()
    assert isinstance(sa.choose(2 ** 16), Float16Compression) and isinstance(sa.choose(2 ** 16 + 1), Uniform8BitQuantization)
    assert shard_bounds(10, [1, 0, 1]) == [0, 5, 5, 10]


def test_dht_store_get_and_expiration():
    from dalle_amd.parallel.dht import DHT, get_dht_time

    d1 = DHT(start=True, host_maddrs=["/ip4/127.0.0.1/tcp/0"])
    d2 = DHT(start=True, initial_peers=d1.get_visible_maddrs())
    now = get_dht_time()
    assert d1.store("run_metrics", subkey=b"peerA", value={"step": 1, "loss": 2.0}, expiration_time=now + 30)
    fut = d2.store("run_metrics", subkey=b"peerB", value={"step": 1, "loss": 3.0}, expiration_time=now + 30, return_future=True)
    assert fut.result()
    d2.store("short", subkey=b"x", value=1, expiration_time=now + 0.2)
    got = d1.get("run_metrics", latest=True)
    assert set(got.value.keys()) == {b"peerA", b"peerB"}
    assert got.value[b"peerB"].value["loss"] == 3.0
    # owner-tagged subkeys: peer 2 cannot overwrite peer 1's live record
    assert not d2.store("run_metrics", subkey=b"peerA", value={"step": 9}, expiration_time=now + 60)
    time.sleep(0.3)
    assert d1.get("short") is None
    assert d2.wait_for("run_metrics", 2, 0.5) == 2
    d2.shutdown()
    d1.shutdown()
