"""Elastic membership: survivors re-form the group after a peer dies; a late joiner is
admitted at the next global step and brought to the collaboration's state by a donor."""
import os
import pickle
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q, die_after, start_delay, min_peers, epochs, want_world, stall_at=0, timeout=20.0):
    try:
        torch.set_num_threads(1)
        time.sleep(start_delay)
        from dalle_amd.parallel.elastic import ElasticGroup, coordinator_store
        from dalle_amd.parallel.optimizer import CollaborativeOptimizer

        store = coordinator_store("127.0.0.1", port, is_master=False, timeout=60)
        eg = ElasticGroup(store, peer_id=f"p{rank}", matchmaking_time=1.0, allreduce_timeout=timeout, min_peers=min_peers)
        eg.join()
        p = torch.nn.Parameter(torch.zeros(32))
        opt = CollaborativeOptimizer(run_id="el", params=[p], optimizer=lambda ps: torch.optim.SGD(ps, lr=0.1),
                                     target_batch_size=4, batch_size_per_step=1, reuse_grad_buffers=True,
                                     average_state_every=0, elastic=eg)
        steps = 0
        # a late joiner's state arrives with the regroup's donor broadcast
        while opt.local_epoch < epochs or eg.world_size < want_world:
            time.sleep(0.02)
            g = torch.full_like(p, float(rank + 1))
            p.grad = g.clone() if p.grad is None else p.grad.add_(g)
            opt.step()
            steps += 1
            if die_after and steps == die_after:
                os._exit(0)  # abrupt death: no goodbye to the group
            if stall_at and steps == stall_at:
                time.sleep(3 * timeout)  # a straggler far past allreduce_timeout
            if steps > 1500:
                raise RuntimeError("no progress")
        q.put(pickle.dumps((rank, eg.world_size, eg.generation, eg.regroups, opt.local_epoch, p.detach().clone())))
        eg.shutdown()
    except Exception:  # pragma: no cover
        import traceback

        q.put(pickle.dumps(("error", rank, traceback.format_exc())))


def _run(specs, expect):
    import torch.distributed as dist

    port = _free_port()
    server = dist.TCPStore("127.0.0.1", port, world_size=None, is_master=True, wait_for_workers=False)
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    procs = [ctx.Process(target=_worker, args=(r, port) + (q,) + spec) for r, spec in enumerate(specs)]
    for pr in procs:
        pr.start()
    res = []
    t0 = time.time()
    while len(res) < expect and time.time() - t0 < 150:
        if not q.empty():
            res.append(pickle.loads(q.get()))
        else:
            time.sleep(0.1)
    for pr in procs:
        pr.join(20)
        if pr.is_alive():
            pr.kill()
    del server
    for r in res:
        assert r[0] != "error", r[2]
    assert len(res) == expect, "elastic peers did not finish"
    return sorted(res, key=lambda r: r[0])


@pytest.mark.slow
def test_survivors_regroup_after_peer_death():
    # (die_after, start_delay, min_peers, epochs, want_world)
    specs = [(0, 0.0, 3, 4, 1), (0, 0.0, 3, 4, 1), (3, 0.0, 3, 4, 1)]
    res = _run(specs, expect=2)
    (r0, w0, g0, n0, e0, p0), (r1, w1, g1, n1, e1, p1) = res
    assert w0 == w1 == 2 and g0 == g1 >= 1 and n0 >= 1
    assert torch.allclose(p0, p1)


@pytest.mark.slow
def test_late_joiner_is_admitted_and_synced():
    specs = [(0, 0.0, 2, 5, 3), (0, 0.0, 2, 5, 3), (0, 4.0, 2, 5, 3)]
    res = _run(specs, expect=3)
    worlds = {r[1] for r in res}
    assert worlds == {3}
    ps = [r[5] for r in res]
    assert torch.allclose(ps[0], ps[1]) and torch.allclose(ps[0], ps[2])


@pytest.mark.slow
def test_straggler_past_timeout_is_dropped_then_readmitted():
    # (die_after, start_delay, min_peers, epochs, want_world, stall_at, timeout)
    specs = [(0, 0.0, 3, 6, 3, 0, 3.0), (0, 0.0, 3, 6, 3, 0, 3.0), (0, 0.0, 3, 6, 3, 3, 3.0)]
    res = _run(specs, expect=3)
    assert {r[1] for r in res} == {3}
    assert all(r[3] >= 1 for r in res)  # everybody regrouped at least once
    ps = [r[5] for r in res]
    assert torch.allclose(ps[0], ps[1]) and torch.allclose(ps[0], ps[2])


def test_recovery_store_is_namespaced_per_torchrun_attempt(monkeypatch):
    """torchrun --max-restarts restarts every worker against the SAME agent store: each attempt's
    generations live under their own prefix, so a restarted world never sees the previous one's keys."""
    import datetime
    import socket

    import torch.distributed as dist

    from dalle_amd.parallel.elastic import recovery_store

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    agent = dist.TCPStore("127.0.0.1", port, world_size=None, is_master=True, timeout=datetime.timedelta(seconds=10),
                          wait_for_workers=False)
    monkeypatch.delenv("DALLE_AMD_COORDINATOR", raising=False)
    monkeypatch.setenv("TORCHELASTIC_USE_AGENT_STORE", "True")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(port))
    for attempt in ("0", "2"):
        monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", attempt)
        recovery_store("job", timeout=10).set("elastic/gen", attempt)
    assert agent.get("dalle_recovery/job/elastic/gen") == b"0"
    assert agent.get("dalle_recovery/job/attempt2/elastic/gen") == b"2"
