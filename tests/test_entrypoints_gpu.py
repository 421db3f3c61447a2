"""run_trainer.py on MI355X: the collaborative training loop end to end on the GPU path (fused HIP
sublayers, fused 8-bit LAMB on the flat arena, delayed optimizer step on a side HIP stream as
task.py configures it). One peer over RCCL, and two peers sharing the card over gloo."""
import os
import re
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COMMON = ["--model_preset", "tiny", "--text_seq_length", "64", "--authorize", "False", "--experiment_prefix", "gpu",
          "--dataloader_num_workers", "0", "--per_device_train_batch_size", "4", "--warmup_steps", "1",
          "--total_steps", "50"]


def _port():
    """A free port whose successor is free too (run_trainer's key-value store binds MASTER_PORT + 1)."""
    for _ in range(50):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        s2 = socket.socket()
        try:
            s2.bind(("127.0.0.1", p + 1))
            return p
        except OSError:
            continue
        finally:
            s2.close()
    raise RuntimeError("no free port pair")


def _run(tmp_path, nproc, extra, timeout=110):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", DALLE_AMD_LOGLEVEL="INFO")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "run_trainer.py"), *COMMON,
           "--output_dir", str(tmp_path / "out"), *extra]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:]
    return r.stdout


def test_single_peer_rccl(cuda, tmp_path):
    out = _run(tmp_path, 1, ["--target_batch_size", "8", "--max_steps", "12"])
    epochs = [int(m) for m in re.findall(r"epoch (\d+): contributed", out)]
    assert epochs and max(epochs) >= 5, out[-3000:]
    assert "cuda" in out
    # the delayed step runs LAMB over the master copies: the fused HIP engine, never the per-tensor path
    assert "LAMB: fused HIP engine over the flat arena" in out, out[-3000:]
    assert "per-tensor PyTorch path" not in out


def test_two_peers_share_the_gpu_over_gloo(cuda, tmp_path):
    out = _run(tmp_path, 2, ["--backend", "gloo", "--target_batch_size", "16", "--max_steps", "8"])
    # asynchronous progress: each round averages at least the target (a peer may add one more micro-batch)
    totals = [int(m) for m in re.findall(r"averaged (\d+) samples across 2 peers", out)]
    assert totals and all(16 <= t <= 16 + 2 * 4 for t in totals), out[-3000:]
    assert "aborting the communicator" not in out
