"""The RCCL communicator lifecycle the failure path relies on, executed on a real MI355X:
form an ``ElasticGroup`` generation over the ``nccl`` (= RCCL) backend, run guarded collectives, wait on
them under a host ``Deadline`` (``watchdog.wait_device``), ABORT the communicator (``ncclCommAbort`` via
``watchdog.abort_group`` inside ``regroup()``) and re-form the next generation on a fresh communicator.

One rank: RCCL refuses two ranks on one device (profiles/r3_rccl_shared_gpu_probe.txt), so the multi-peer
failure cases run on gloo (tests/test_elastic_cpu.py); what this adds is that the abort and re-init calls
themselves work against RCCL -- until now they had only ever run on gloo. Runs in a child process so the
default process group never leaks into the pytest process."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import datetime, json, sys, time
import torch, torch.distributed as dist
sys.path.insert(0, sys.argv[2])
from dalle_amd.parallel.elastic import ElasticGroup, coordinator_store
from dalle_amd.parallel.watchdog import Deadline, wait_device

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
store = coordinator_store("127.0.0.1", int(sys.argv[1]), is_master=True, timeout=60)
eg = ElasticGroup(store, "p0", backend="nccl", matchmaking_time=0.2, allreduce_timeout=30.0, device=dev)
res = {"generations": [], "values": [], "backend": []}
eg.join()
for step in range(3):
    x = torch.full((1 << 20,), float(step + 1), device=dev)
    eg.guarded(lambda: dist.all_reduce(x, async_op=True))
    wait_device(dev, Deadline(30.0), "all_reduce")
    res["values"].append(float(x[0].item()))
    res["generations"].append(eg.generation)
    res["backend"].append(dist.get_backend())
    res["join_flag"] = eg.poll_join()
    if step < 2:
        eg.regroup()  # ncclCommAbort on the live communicator, then generation g + 1 on a new one
res["regroups"] = eg.regroups
eg.shutdown()
print("RESULT " + json.dumps(res), flush=True)
"""


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_rccl_abort_and_reform_generations():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR")}
    out = subprocess.run([sys.executable, "-c", CHILD, str(_port()), ROOT], env=env, capture_output=True, text=True,
                         timeout=100)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("RESULT ")]
    assert line, out.stdout[-2000:] + out.stderr[-2000:]
    res = json.loads(line[0][len("RESULT "):])
    assert res["backend"] == ["nccl"] * 3
    assert res["generations"] == [0, 1, 2] and res["regroups"] == 2
    assert res["values"] == [1.0, 2.0, 3.0]  # world of one: the sum is the tensor itself
    assert res["join_flag"] is False
