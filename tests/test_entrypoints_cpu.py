"""BASELINE config 1 on CPU: tiny DALL-E, two run_trainer.py peers (torchrun, gloo) + an aux peer
that reads their metrics from the key-value store and snapshots the training state."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    for _ in range(50):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        s2 = socket.socket()
        try:
            s2.bind(("127.0.0.1", p + 1))
            s2.close()
            return p
        except OSError:
            s2.close()
    raise RuntimeError("no free port pair")


COMMON = ["--model_preset", "tiny", "--text_seq_length", "64", "--authorize", "False", "--experiment_prefix", "cfg1",
          "--dataloader_num_workers", "0"]


@pytest.mark.slow
def test_two_peers_plus_aux(tmp_path):
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", DALLE_AMD_LOGLEVEL="INFO")
    out = tmp_path / "out"
    trainer = subprocess.Popen(
        [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
         "--master-port", str(port), os.path.join(ROOT, "run_trainer.py"), *COMMON, "--per_device_train_batch_size", "2",
         "--target_batch_size", "8", "--max_steps", "120", "--warmup_steps", "2", "--total_steps", "100",
         "--output_dir", str(out), "--backup_every_steps", "2", "--state_path", str(tmp_path / "state.zip")],
        cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    time.sleep(8)
    metrics_log = tmp_path / "metrics.jsonl"
    aux = subprocess.run(
        [sys.executable, os.path.join(ROOT, "run_aux_peer.py"), *COMMON, "--initial_peers", f"/ip4/127.0.0.1/tcp/{port + 1}",
         "--refresh_period", "0.5", "--max_iterations", "14", "--metrics_log", str(metrics_log),
         "--save_checkpoint_step_interval", "2", "--local_path", str(tmp_path / "repo"), "--output_dir", str(tmp_path / "aux")],
        cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240)
    try:
        tout, _ = trainer.communicate(timeout=300)
    except subprocess.TimeoutExpired:
        trainer.kill()
        raise
    assert trainer.returncode == 0, tout[-4000:]
    assert aux.returncode == 0, aux.stdout[-4000:]
    # 2 peers x 2 samples per step, target 8 -> an epoch every ~2 local steps per peer (asynchronous
    # progress: a peer may add one more micro-batch before it notices the target was reached)
    import re
    assert re.search(r"cfg1: epoch 5 \(averaged (8|10|12) samples across 2 peers", tout), tout[-3000:]
    assert "aborting the communicator" not in tout, tout[-3000:]
    records = [json.loads(l) for l in metrics_log.read_text().splitlines()]
    assert records and max(r["alive peers"] for r in records) == 2
    # epoch 0 closes on the first micro-step, before the device-timed EMA has an interval: no throughput
    # is reported there (None), a positive one on every later epoch
    assert all(r["performance"] is None for r in records if r["step"] == 0)
    assert all(r["performance"] is not None and r["performance"] > 0 for r in records if r["step"] > 0)
    # the aux peer fetched a state snapshot from the group and wrote reference-format checkpoints
    assert (tmp_path / "repo" / "model_state.pt").exists()
    sd = torch.load(tmp_path / "repo" / "model_state.pt", weights_only=True)
    assert "model.to_logits.1.weight" in sd
    osd = torch.load(tmp_path / "repo" / "optimizer_state.pt", weights_only=True)
    assert "local_epoch" in osd["state"]
    # backups written by the training callback
    st = torch.load(tmp_path / "state.rank0.zip", weights_only=True)  # one backup file per peer
    assert (tmp_path / "state.rank1.zip").exists()
    assert set(st) == {"model", "training", "scheduler", "local_epoch"}


def test_nan_rollback_and_averaging_fallback(tmp_path):
    """Fault injection (SURVEY §4 tier 5): NaN parameters after epoch 3 -> the callback restores the
    backup; an injected averaging failure at epoch 1 -> local gradients are used and training goes on."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", DALLE_AMD_FAULT_NAN_PARAMS="3",
               DALLE_AMD_FAULT_FAIL_AVERAGING="1")
    r = subprocess.run(
        [sys.executable, os.path.join(ROOT, "run_trainer.py"), *COMMON, "--per_device_train_batch_size", "2",
         "--target_batch_size", "2", "--max_steps", "6", "--warmup_steps", "1", "--total_steps", "10",
         "--output_dir", str(tmp_path / "out"), "--backup_every_steps", "1", "--state_path", str(tmp_path / "state.zip")],
        cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-4000:]
    assert "falling back to local gradients" in r.stdout
    assert "Parameters became NaN/Inf: rolling back to the last backup" in r.stdout
    assert "Restored the backup of epoch" in r.stdout


@pytest.mark.slow
def test_torchrun_restart_resumes_from_backups_and_donor(tmp_path):
    """torchrun --max-restarts 1: rank 1 dies at epoch 3 of the first attempt; the agent restarts the whole
    world, every peer restores its own backup, then synchronises with the donor (load_state_from_peers), and
    the two peers go on averaging together past the failure."""
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", DALLE_AMD_LOGLEVEL="INFO",
               DALLE_AMD_FAULT_KILL_AT_EPOCH="3", DALLE_AMD_FAULT_RANK="1", DALLE_AMD_FAULT_ATTEMPT="0")
    out = tmp_path / "out"
    run = subprocess.run(
        [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2", "--max-restarts", "1",
         "--monitor-interval", "0.5", "--master-addr", "127.0.0.1", "--master-port", str(port),
         os.path.join(ROOT, "run_trainer.py"), *COMMON, "--per_device_train_batch_size", "2", "--target_batch_size", "8",
         "--max_steps", "24", "--warmup_steps", "2", "--total_steps", "100", "--output_dir", str(out),
         "--backup_every_steps", "1", "--state_path", str(tmp_path / "state.zip"), "--averaging_timeout", "60"],
        cwd=tmp_path, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    tout = run.stdout
    assert run.returncode == 0, tout[-4000:]
    assert tout.count("Restored the backup of epoch") >= 2, tout[-4000:]  # both restarted peers
    import re
    after = [int(m) for m in re.findall(r"cfg1: epoch (\d+) \(averaged \d+ samples across 2 peers", tout)]
    assert sum(e >= 6 for e in after) >= 4, tout[-3000:]  # both peers, several rounds past the restart
    for r in (0, 1):
        assert torch.load(tmp_path / f"state.rank{r}.zip", weights_only=True)["local_epoch"] >= 6
