"""bench.py's multi-rank contract on CPU (gloo): ``--gpus N`` without a launcher spawns N ranks,
each asserts the group size, the ranks stay bitwise identical, and only rank 0 prints one JSON line."""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, *extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(BENCH_BACKEND="gloo", BENCH_DUMP_PARAMS=str(tmp_path / "params"), HIP_VISIBLE_DEVICES="")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
                          "--model", "tiny", "--batch", "2", *extra], env=env, cwd=str(tmp_path), capture_output=True,
                         text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    p0 = torch.load(tmp_path / "params.rank0.pt", weights_only=True)
    p1 = torch.load(tmp_path / "params.rank1.pt", weights_only=True)
    return res, p0, p1


@pytest.mark.parametrize("engine", ["step", "collab"])
def test_bench_spawns_n_ranks(tmp_path, engine):
    res, p0, p1 = _run(tmp_path, "--engine", engine)
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2" and res["config"]["global_batch"] == 4
    assert len(res["per_rank_ms_per_step"]) == 2 and res["value"] > 0
    assert len(res["per_rank_peak_mem_gb"]) == 2
    if engine == "step":  # the gradient all-reduce priced inside the run (bytes, bus bandwidth, overlap)
        ar = res["grad_allreduce"]
        assert ar["bytes_per_step"] > 0 and ar["busbw_GBps"] > 0 and ar["standalone_ms"] > 0
        assert 0.0 <= ar["overlapped_frac"] <= 1.0
        # --allreduce-algo / --bucket-mb auto: every (algorithm, bucket) candidate timed on the real communicator
        # at start-up, the fastest selected -- the same on every rank (the params below stay bitwise identical)
        sel, table = ar["selected"], ar["tuning"]
        assert sel["tuned"] and len(table) == 8 and {r["algo"] for r in table} == {"rccl", "rs_ag"}
        # the 3 standalone winners re-timed inside a real step (backward hand-off attached); selected on that
        stepped = [r for r in table if r["step_ms"] is not None]
        top3 = sorted(table, key=lambda r: (r["ms"], r["algo"], r["bucket_mb"]))[:3]
        assert len(stepped) == 3 and all(r in top3 for r in stepped) and all(r["step_ms"] > 0 for r in stepped)
        best = min(stepped, key=lambda r: (r["step_ms"], r["algo"], r["bucket_mb"]))
        assert (sel["algo"], sel["bucket_mb"]) == (best["algo"], best["bucket_mb"]) == (ar["algo"], sel["bucket_mb"])
    assert torch.equal(p0, p1)  # replicas stay bitwise identical
    if engine == "collab":
        assert res["config"]["engine"] == "CollaborativeOptimizer.step"
        assert res["collab_performance_ema_samples_per_s"] > 0
        # static homogeneous peers, uncompressed: every round is the backward-armed GradSync path
        assert res["collab_backward_overlapped_rounds"] >= 3


@pytest.mark.parametrize("n", [2, 4])
def test_bench_allreduce_algorithms(tmp_path, n):
    """--allreduce-algo rs_ag (bucketed reduce-scatter + all-gather) against the plain all_reduce: every
    rank bitwise identical under both; at 2 ranks the two algorithms agree bitwise (one add per element),
    at 4 to rounding (a different reduction order); the JSON names the algorithm and prices every bucket."""
    outs = {}
    for algo in ("rccl", "rs_ag"):
        d = tmp_path / algo
        d.mkdir()
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
        env.update(BENCH_BACKEND="gloo", BENCH_DUMP_PARAMS=str(d / "params"), HIP_VISIBLE_DEVICES="")
        out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "2", "--warmup", "1",
                              "--model", "tiny", "--batch", "2", "--allreduce-algo", algo], env=env, cwd=str(d),
                             capture_output=True, text=True, timeout=600)
        assert out.returncode == 0, out.stderr[-3000:]
        res = json.loads([ln for ln in out.stdout.splitlines() if ln.startswith("{")][0])
        assert res["config"]["grad_allreduce_algo"] == algo and res["grad_allreduce"]["algo"] == algo
        assert res["grad_allreduce"]["buckets"] and all(b["busbw_GBps"] > 0 for b in res["grad_allreduce"]["buckets"])
        ps = [torch.load(d / f"params.rank{r}.pt", weights_only=True) for r in range(n)]
        assert all(torch.equal(ps[0], p) for p in ps[1:])
        outs[algo] = ps[0]
    if n == 2:
        assert torch.equal(outs["rccl"], outs["rs_ag"])
    else:
        assert torch.allclose(outs["rccl"], outs["rs_ag"], rtol=1e-5, atol=1e-6)


def test_bench_rejects_world_mismatch(tmp_path):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", BENCH_BACKEND="gloo", HIP_VISIBLE_DEVICES="")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "tiny"], env=env,
                         cwd=str(tmp_path), capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "WORLD_SIZE=1" in out.stderr


@pytest.mark.parametrize("n", [2, 4])
def test_bench_under_torchrun(tmp_path, n):
    """The driver's multi-GPU form: ``torch.distributed.run --nproc-per-node N ... bench.py --gpus N`` (here
    with gloo on CPU): the launcher's ranks are used as they are (no second spawn), one JSON line, every
    rank's parameters bitwise identical after the steps."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(BENCH_BACKEND="gloo", BENCH_DUMP_PARAMS=str(tmp_path / "params"), HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "2", "--warmup", "1",
           "--model", "tiny", "--batch", "2"]
    out = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == n and res["backend"] == "gloo" and len(res["per_rank_ms_per_step"]) == n
    assert res["config"]["parallelism"] == f"dp{n}" and res["config"]["global_batch"] == 2 * n
    ps = [torch.load(tmp_path / f"params.rank{r}.pt", weights_only=True) for r in range(n)]
    assert all(torch.equal(ps[0], p) for p in ps[1:])


def test_bench_bf16_wire(tmp_path):
    """--grad-dtype bf16 with a fixed bucket and algorithm (no tuning): ranks stay bitwise identical (the
    hand-over from inside backward is covered by tests/test_dp_cpu.py)."""
    res, p0, p1 = _run(tmp_path, "--grad-dtype", "bf16", "--allreduce-algo", "rs_ag", "--bucket-mb", "1")
    ar = res["grad_allreduce"]
    assert res["config"]["grad_allreduce_dtype"] == "bf16" and ar["selected"]["bucket_mb"] == 1.0
    assert not ar["selected"]["tuned"] and ar["tuning"] is None
    assert torch.equal(p0, p1)


def test_bench_fixed_bucket_with_auto_algorithm(tmp_path):
    """--bucket-mb fixed, --allreduce-algo auto: only the algorithm is tuned, at that (integer-byte) bucket."""
    res, p0, p1 = _run(tmp_path, "--bucket-mb", "1")
    ar = res["grad_allreduce"]
    assert ar["selected"]["tuned"] and ar["selected"]["bucket_mb"] == 1.0
    assert sorted(r["algo"] for r in ar["tuning"]) == ["rccl", "rs_ag"]
    assert torch.equal(p0, p1)


@pytest.mark.parametrize("algo,dtype", [("rs_ag", "bf16"), ("rccl", "fp32")])
def test_bench_world8(tmp_path, algo, dtype):
    """8 ranks -- the MI355X node's world -- through bench.py's own spawn: one JSON line, dp8, every rank's
    parameters bitwise identical after the steps."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(BENCH_BACKEND="gloo", BENCH_DUMP_PARAMS=str(tmp_path / "params"), HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "2", "--warmup", "1",
                          "--model", "tiny", "--batch", "1", "--allreduce-algo", algo, "--grad-dtype", dtype,
                          "--bucket-mb", "1"], env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 8 and res["config"]["parallelism"] == "dp8" and res["config"]["global_batch"] == 8
    assert res["grad_allreduce"]["algo"] == algo and res["config"]["grad_allreduce_dtype"] == dtype
    ps = [torch.load(tmp_path / f"params.rank{r}.pt", weights_only=True) for r in range(8)]
    assert all(torch.equal(ps[0], p) for p in ps[1:])
