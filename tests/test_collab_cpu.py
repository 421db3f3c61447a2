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
    # asynchronous progress: each peer contributes at its own pace; the epoch closes once the shared
    # counter reaches the target (overshoot < one step of each peer), weights are the exact counts
    assert s0 + s1 >= 16 and s0 + s1 < 16 + 3 + 5
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


# ------------------------------------------------------------------------------------------------
def _mixed_scale_worker(rank, world, port, q):
    """State averaging of an arena whose tensors differ in scale by 4 orders of magnitude: every
    tensor must be compressed on its own (fp16 below 2^16+1 elements, 8-bit per 2^17-element part
    above), so small-scale tensors survive the round (one codebook for the whole arena
    erased them)."""
    try:
        _init(rank, world, port)
        from dalle_amd.optim import FlatArena
        from dalle_amd.parallel.averaging import allreduce_weighted

        g = torch.Generator().manual_seed(100 + rank)
        shapes_scales = [((300, 1000), 1.0), ((1000,), 1e-3), ((70, 1000), 1e-4), ((64,), 3e-5), ((4, 3001), 0.2)]
        params = [torch.nn.Parameter(torch.randn(*s, generator=g) * sc) for s, sc in shapes_scales]
        arena = FlatArena(params)
        before = [p.detach().clone() for p in params]
        allreduce_weighted(arena.data, 1.0, compression=reference_averaging_compression(), total_weight=float(world),
                           segments=arena.segments())
        q.put(pickle.dumps((rank, before, [p.detach().clone() for p in params])))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_butterfly_compresses_each_tensor_separately():
    (r0, b0, a0), (r1, b1, a1) = _run(_mixed_scale_worker, 2)
    for i, (x0, x1, y0, y1) in enumerate(zip(b0, b1, a0, a1)):
        exact = (x0 + x1) / 2
        assert torch.equal(y0, y1), i  # every peer extracts the same averaged values
        rel = ((y0 - exact).norm() / exact.norm()).item()
        limit = 3e-3 if exact.numel() < 2 ** 16 + 1 else 0.04  # fp16 (subnormal below 6e-5) vs uniform 8-bit
        assert rel < limit, (i, rel)


# ------------------------------------------------------------------------------------------------
def _speed_worker(rank, world, port, q, nap):
    try:
        _init(rank, world, port)
        from dalle_amd.parallel.optimizer import CollaborativeOptimizer

        p = torch.nn.Parameter(torch.zeros(1000))
        p.grad = torch.zeros_like(p)
        opt = CollaborativeOptimizer(run_id="speed", params=[p], optimizer=lambda ps: torch.optim.SGD(ps, lr=0.1),
                                     target_batch_size=60, batch_size_per_step=1, reuse_grad_buffers=True)
        assert opt.tracker.mode == "store"
        dist.barrier()  # both peers start together (process start-up skew is not a speed difference)
        steps = 0
        while opt.local_epoch == 0:
            time.sleep(nap[rank])
            p.grad.add_(1.0)
            steps += 1
            opt.step()
        q.put(pickle.dumps((rank, steps)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_heterogeneous_peers_contribute_at_their_own_pace():
    """Peers with a 2:1 speed ratio contribute about 2:1 samples to one epoch (no lockstep)."""
    (r0, n0), (r1, n1) = _run(_speed_worker, 2, (0.01, 0.02))
    assert 60 <= n0 + n1 <= 62
    assert 1.3 < n0 / n1 < 3.2, (n0, n1)


# ------------------------------------------------------------------------------------------------
def _dead_peer_worker(rank, world, port, q, recovery, coord_port, epochs=4):
    try:
        if rank == 2:
            os.environ["DALLE_AMD_FAULT_KILL_IN_AVERAGING"] = "1"
        if coord_port:
            os.environ["DALLE_AMD_COORDINATOR"] = f"127.0.0.1:{coord_port}"
        _init(rank, world, port)
        from dalle_amd.parallel.optimizer import CollaborativeOptimizer

        torch.manual_seed(0)
        p = torch.nn.Parameter(torch.zeros(300, 300))
        p.grad = torch.zeros_like(p)
        opt = CollaborativeOptimizer(run_id="dead", params=[p], optimizer=lambda ps: torch.optim.SGD(ps, lr=1.0),
                                     target_batch_size=3, batch_size_per_step=1, reuse_grad_buffers=True,
                                     averaging_timeout=20.0, allreduce_timeout=10.0, matchmaking_time=1.0,
                                     tracker_mode="static", recovery=recovery)
        epochs_grads = []
        while opt.local_epoch < epochs:
            g = torch.full_like(p, float(rank + 1) * (opt.local_epoch + 1))
            p.grad.add_(g)
            before = p.detach().clone()
            e = opt.local_epoch
            opt.step()
            epochs_grads.append((e, (before - p.detach()).mean().item()))
        regroups = opt.elastic.regroups if opt.elastic is not None else 0
        world_after = opt.elastic.world_size if opt.elastic is not None else 1
        q.put(pickle.dumps((rank, opt.detached, epochs_grads, p.detach().clone(), regroups, world_after)))
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def _joiner_worker(coord_port, q):
    """A replacement peer: joins the survivors' group through the coordinator, gets the state from a donor
    and trains on with them."""
    try:
        os.environ["DALLE_AMD_COORDINATOR"] = f"127.0.0.1:{coord_port}"
        torch.set_num_threads(1)
        import datetime

        from dalle_amd.parallel.elastic import ElasticGroup, recovery_store
        from dalle_amd.parallel.optimizer import CollaborativeOptimizer

        store = recovery_store("dead")
        store.wait(["elastic/g0/frozen"], datetime.timedelta(seconds=120))  # the survivors regrouped once
        eg = ElasticGroup(store, peer_id="joiner", backend="gloo", matchmaking_time=1.0, allreduce_timeout=10.0)
        eg.join()
        p = torch.nn.Parameter(torch.full((300, 300), 123.0))  # garbage until the donor's state arrives
        p.grad = torch.zeros_like(p)
        opt = CollaborativeOptimizer(run_id="dead", params=[p], optimizer=lambda ps: torch.optim.SGD(ps, lr=1.0),
                                     target_batch_size=3, batch_size_per_step=1, reuse_grad_buffers=True,
                                     averaging_timeout=20.0, allreduce_timeout=10.0, matchmaking_time=1.0, elastic=eg)
        assert opt.tracker.mode == "static", opt.tracker.mode  # the adopted group's published mode
        opt.load_state_from_peers()  # pairs with the members' regroup-time resync
        joined_at = opt.local_epoch
        while opt.local_epoch < 6:
            p.grad.add_(3.0 * (opt.local_epoch + 1))
            opt.step()
        q.put(pickle.dumps(("joiner", joined_at, p.detach().clone(), eg.world_size)))
        eg.shutdown()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", "joiner", traceback.format_exc())))


def _run_with_dead_peer(recovery, coordinator, epochs=4, joiner=False):
    port = _free_port()
    server = None
    coord_port = 0
    if coordinator:  # a store that outlives every trainer (the torchrun agent's role)
        coord_port = _free_port()
        server = dist.TCPStore("127.0.0.1", coord_port, world_size=None, is_master=True, wait_for_workers=False)
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_dead_peer_worker, args=(r, 3, port, q, recovery, coord_port, epochs)) for r in range(3)]
    if joiner:
        procs.append(ctx.Process(target=_joiner_worker, args=(coord_port, q)))
    for p in procs:
        p.start()
    res = sorted([pickle.loads(q.get()) for _ in range(2 + int(joiner))], key=lambda r: str(r[0]))
    for p in procs:
        p.join(60)
        if p.is_alive():
            p.kill()
    del server
    for r in res:
        assert r[0] != "error", r[2]
    return res


def test_dead_peer_survivors_regroup_and_keep_averaging():
    """Default path with a store that outlives the trainers: a rank SIGKILLed inside the epoch-1 averaging
    round. The survivors' round fails (each applies its own gradient), they abort the communicator,
    re-form a 2-peer group, sync from the donor (rank 0) and average WITH EACH OTHER from epoch 2 on."""
    res = _run_with_dead_peer("auto", coordinator=True)
    (_, d0, s0, p0, n0, w0), (_, d1, s1, p1, n1, w1) = res
    assert not d0 and not d1
    assert n0 == n1 == 1 and w0 == w1 == 2
    assert torch.equal(p0, p1)
    u0, u1 = dict(s0), dict(s1)
    for upd in (u0, u1):
        assert abs(upd[0] - 2.0) < 1e-5, upd            # 3 peers: (1 + 2 + 3) / 3
        # failed round: each survivor applied its own gradient, then the new group synced from its donor
        assert min(abs(upd[1] - 2.0), abs(upd[1] - 4.0)) < 1e-5, upd
        assert abs(upd[2] - 1.5 * 3) < 1e-5, upd        # 2 peers: (1 + 2) / 2 * (e + 1)
        assert abs(upd[3] - 1.5 * 4) < 1e-5, upd
    assert u0[1] == u1[1]


def test_replacement_peer_joins_survivors_and_gets_state_from_donor():
    """After the survivors re-formed their group, a replacement peer joins through the same coordinator: the
    members admit it at their next round boundary, it receives parameters / epoch from a donor, and from
    then on the three train in lockstep (bitwise identical parameters)."""
    res = _run_with_dead_peer("auto", coordinator=True, epochs=6, joiner=True)
    for r in res:
        assert r[0] != "error", r[2]
    (r0, d0, s0, p0, n0, w0), (r1, d1, s1, p1, n1, w1), (_, joined_at, pj, wj) = res
    assert not d0 and not d1 and w0 == w1 == wj == 3
    assert n0 == n1 == 2  # death, then the join
    assert 2 <= joined_at < 6
    assert torch.equal(p0, p1) and torch.equal(p0, pj)


def test_dead_peer_without_recovery_store_detaches():
    """recovery="detach" (or no store that outlives the trainers): the survivors abort the communicator,
    apply their OWN gradients for that epoch and keep training alone."""
    res = _run_with_dead_peer("detach", coordinator=False)
    for rank, detached, steps, _, _, _ in res:
        assert detached
        upd = dict(steps)
        assert abs(upd[0] - 2.0) < 1e-5, upd
        assert abs(upd[1] - (rank + 1) * 2.0) < 1e-5, upd
        assert abs(upd[3] - (rank + 1) * 4.0) < 1e-5, upd


# ------------------------------------------------------------------------------------------------
def _lagging_collective_worker(rank, world, port, q):
    """Lockstep ("collective") tracker with one peer two epochs behind (e.g. it restored an old local
    backup): the resync is a collective, so EVERY rank must take it -- the laggard as receiver, the
    others as donors -- or the group deadlocks on mismatched collectives."""
    try:
        _init(rank, world, port)
        from dalle_amd.parallel.optimizer import CollaborativeOptimizer

        torch.manual_seed(rank)
        p = torch.nn.Parameter(torch.randn(50, 40))
        opt = CollaborativeOptimizer(run_id="lag", params=[p], optimizer=lambda ps: torch.optim.SGD(ps, lr=0.1),
                                     target_batch_size=4, batch_size_per_step=2, reuse_grad_buffers=True,
                                     average_state_every=0, tracker_mode="collective")
        opt.local_epoch = 5 if rank == 0 else 2
        opt.tracker.update_epoch(opt.local_epoch)
        p.grad = torch.ones_like(p)
        opt.step()
        q.put(pickle.dumps((rank, opt.local_epoch, p.detach().clone())))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def test_collective_tracker_resyncs_lagging_peer_on_every_rank():
    (r0, e0, p0), (r1, e1, p1) = _run(_lagging_collective_worker, 2)
    assert e0 == e1 == 5
    assert torch.equal(p0, p1)
