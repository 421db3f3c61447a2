"""Multi-GPU data parallelism over RCCL (SURVEY §4 tier 6): ``torchrun --nproc-per-node N bench.py --gpus N``
-- the driver's scaling launch -- with the gradient all-reduce handed off during backward and without.
Runs only where at least two GPUs are visible: RCCL refuses two ranks on one device ("Duplicate GPU detected",
profiles/r3_rccl_shared_gpu_probe.txt), so it is skipped on a one-GPU box; the same path is rehearsed there
with gloo, tests/test_bench_cpu.py and scripts/gpu_handoff.sh)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NGPU = torch.cuda.device_count()


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(tmp_path, n, overlap):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(DALLE_AMD_DP_OVERLAP=str(overlap), BENCH_DUMP_PARAMS=str(tmp_path / f"p{overlap}"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "2",
           "--warmup", "1", "--batch", "8"]
    out = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=400)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0]), [torch.load(tmp_path / f"p{overlap}.rank{r}.pt", weights_only=True) for r in range(n)]


@pytest.mark.skipif(NGPU < 2, reason="needs at least two GPUs")
def test_rccl_data_parallel_ranks_identical_with_and_without_handoff(tmp_path):
    n = min(NGPU, 8)
    res1, p1 = _torchrun(tmp_path, n, 1)
    res0, p0 = _torchrun(tmp_path, n, 0)
    assert res1["n_gpus"] == n and res1["rccl_world"] == n and len(set(res1["devices"])) >= 1
    assert res1["grad_allreduce_overlapped_frac"] > 0.5 and res0["grad_allreduce_overlapped_frac"] == 0.0
    for p in (p0, p1):
        assert all(torch.equal(p[0], q) for q in p[1:])  # every rank holds the same parameters
    # the hand-off only changes how the arena is bucketed on the wire
    assert torch.allclose(p1[0], p0[0], rtol=1e-5, atol=1e-6)
