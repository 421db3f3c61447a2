"""Local swarm manager (the scale-set counterpart): aux peer + elastic trainers as
processes; an evicted trainer is restarted by the supervisor and rejoins the group."""
import glob
import os

import pytest

from dalle_amd.utils.swarm import LocalSwarm, _cli


def test_swarm_commands(tmp_path):
    sw = LocalSwarm(2, peer_args=["--model_preset", "tiny"], log_dir=str(tmp_path), devices=[0, 1])
    aux, t1 = sw.aux_peer(), sw.trainer(1)
    assert "--host_elastic_coordinator" in aux.cmd and f"127.0.0.1:{sw.coordinator_port}" in aux.cmd
    assert f"/ip4/127.0.0.1/tcp/{sw.dht_port}" in t1.cmd and "--elastic_coordinator" in t1.cmd
    assert t1.env["HIP_VISIBLE_DEVICES"] == "1" and "WORLD_SIZE" not in t1.env
    assert _cli(["status", "--log-dir", str(tmp_path / "none")]) == 0


@pytest.mark.slow
def test_evicted_trainer_rejoins(tmp_path):
    common = ["--model_preset", "tiny", "--text_seq_length", "64", "--authorize", "False", "--experiment_prefix", "sw",
              "--dataloader_num_workers", "0", "--output_dir", str(tmp_path / "out")]
    sw = LocalSwarm(2, peer_args=common, log_dir=str(tmp_path / "logs"),
                    trainer_args=["--per_device_train_batch_size", "2", "--target_batch_size", "8", "--max_steps", "100000",
                                  "--warmup_steps", "2", "--total_steps", "100", "--matchmaking_time", "3",
                                  "--allreduce_timeout", "20"], aux_args=["--refresh_period", "1"])
    sw.up()
    try:
        events = sw.supervise(45, chaos_interval=20)
    finally:
        sw.down()
    assert any(e["event"] == "evict" for e in events)
    assert any(e["event"] == "restart" for e in events)
    logs = "".join(open(f).read() for f in glob.glob(os.path.join(str(tmp_path / "logs"), "trainer*.log")))
    assert "regrouping" in logs and "generation 1" in logs
