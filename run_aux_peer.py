#!/usr/bin/env python3
"""Auxiliary peer: collaboration monitor + checkpointer (reference ``run_aux_peer.py:1-152``).

Polls ``{prefix}_metrics`` from the key-value store every ``refresh_period`` seconds, aggregates
loss / alive peers / samples / throughput (Σ samples/s over peers -- the reference's throughput
metric), logs them (wandb when installed, and/or a JSON-lines file), and every
``save_checkpoint_step_interval`` epochs fetches the training state from the peers and writes
``model_state.pt`` / ``optimizer_state.pt`` (pushed to the Hub when ``repo_url`` + ``upload_interval``
are set and ``huggingface_hub`` can reach it).
"""
import json
import os
import time

import torch

import utils
from arguments import AuxiliaryPeerArguments, CollaborativeArguments, HFTrainerArguments
from dalle_amd.parallel.dht import get_dht_time
from dalle_amd.utils.argparse import HfArgumentParser
from dalle_amd.utils.logging import get_logger, use_hivemind_log_handler
from task import TrainingTask

use_hivemind_log_handler("in_root_logger")
logger = get_logger(__name__)


class CheckpointHandler:
    def __init__(self, task: TrainingTask, peer_args: AuxiliaryPeerArguments):
        self.task, self.peer_args = task, peer_args
        self.save_checkpoint_step_interval = peer_args.save_checkpoint_step_interval
        self.prefix = peer_args.experiment_prefix
        self.local_path = peer_args.local_path
        self.upload_interval = peer_args.upload_interval
        self.repo = None
        os.makedirs(self.local_path, exist_ok=True)
        if self.upload_interval is not None and peer_args.repo_url:
            try:
                from huggingface_hub import Repository

                self.repo = Repository(local_dir=self.local_path, clone_from=peer_args.repo_url,
                                       use_auth_token=getattr(task.authorizer, "hf_user_access_token", None))
            except Exception as e:  # noqa: BLE001 - offline: keep checkpoints local
                logger.warning(f"Hub repository unavailable ({e!r}); checkpoints stay in {self.local_path}")
        self.last_upload_time = None
        self.previous_step = -1
        self.local_epoch = 0
        self.optimizer_state = None

    def should_save_state(self, cur_step):
        if self.save_checkpoint_step_interval is None:
            return False
        return cur_step - self.previous_step >= self.save_checkpoint_step_interval

    def load_state_from_peers(self, min_epoch: int, timeout: float = 120.0) -> bool:
        dht = self.task.dht
        dht.store(self.prefix + "_state_request", subkey=dht.peer_id, value=int(min_epoch), expiration_time=get_dht_time() + timeout)
        deadline = time.time() + timeout
        while time.time() < deadline:
            try:
                entry = dht.get(self.prefix + "_state", latest=True)
            except RuntimeError:
                return False
            if entry is not None and int(entry.value["epoch"]) >= min_epoch and os.path.exists(entry.value["path"]):
                state = torch.load(entry.value["path"], map_location="cpu", weights_only=True)
                self.task.model.load_state_dict(state["model"])
                self.optimizer_state = state["optimizer"]
                self.local_epoch = int(state["local_epoch"])
                return True
            time.sleep(0.5)
        logger.warning(f"no peer served a state of epoch >= {min_epoch} within {timeout}s")
        return False

    def save_state(self, cur_step):
        logger.info("Saving state from peers")
        if self.load_state_from_peers(cur_step):
            torch.save(self.task.model.state_dict(), f"{self.local_path}/model_state.pt")
            if self.optimizer_state is not None:
                torch.save(self.optimizer_state, f"{self.local_path}/optimizer_state.pt")
        self.previous_step = cur_step

    def is_time_to_upload(self):
        if self.upload_interval is None:
            return False
        return self.last_upload_time is None or time.time() - self.last_upload_time >= self.upload_interval

    def upload_checkpoint(self, current_loss):
        self.last_upload_time = time.time()
        if self.repo is None:
            return
        logger.info("Started uploading to Model Hub")
        try:
            self.repo.git_pull()
            self.repo.push_to_hub(commit_message=f"Epoch {self.local_epoch}, loss {current_loss:.3f}")
            logger.info("Finished uploading to Model Hub")
        except Exception:  # noqa: BLE001
            logger.exception("Uploading the checkpoint to HF Model Hub failed:")
            logger.warning("Ensure that your access token is valid and has WRITE permissions")


def main(argv=None):
    parser = HfArgumentParser((AuxiliaryPeerArguments, HFTrainerArguments, CollaborativeArguments))
    peer_args, trainer_args, collab_args = parser.parse_args_into_dataclasses(argv)

    coordinator = None
    if peer_args.host_elastic_coordinator and peer_args.elastic_coordinator:
        # the long-lived store elastic trainers rendezvous on: it must outlive every trainer
        from dalle_amd.parallel.elastic import coordinator_store

        host, port = peer_args.elastic_coordinator.rsplit(":", 1)
        coordinator = coordinator_store(host, int(port), is_master=True)
        logger.info(f"hosting the elastic coordinator at {peer_args.elastic_coordinator}")
        peer_args.elastic_coordinator = None  # the aux peer itself is not a trainer / group member

    task = TrainingTask(peer_args, trainer_args, collab_args)
    dht = task.dht

    wandb = None
    if peer_args.wandb_project is not None:
        try:
            import wandb as _wandb

            _wandb.init(project=peer_args.wandb_project)
            wandb = _wandb
        except ImportError:
            logger.warning("wandb is not installed; use --metrics_log for a local JSON-lines log")

    current_step = 0
    checkpoint_handler = CheckpointHandler(task, peer_args) if peer_args.store_checkpoints else None

    if peer_args.assist_in_averaging:
        raise NotImplementedError("aux peers are not members of the RCCL averaging group (same as the reference)")

    iteration = 0
    history = []
    while peer_args.max_iterations is None or iteration < peer_args.max_iterations:
        iteration += 1
        try:
            metrics_entry = dht.get(peer_args.experiment_prefix + "_metrics", latest=True)
        except RuntimeError as e:  # the store's host peer went away
            logger.warning(f"key-value store unreachable ({e}); stopping the monitor")
            break
        if metrics_entry is not None and isinstance(metrics_entry.value, dict) and len(metrics_entry.value) > 0:
            metrics_dict = metrics_entry.value
            metrics = [utils.LocalMetrics.model_validate(metrics_dict[peer].value) for peer in metrics_dict]
            latest_step = max(item.step for item in metrics)

            if latest_step != current_step:
                logger.debug(f"Got metrics from {len(metrics)} peers")
                current_step = latest_step
                alive_peers = 0
                sum_loss = 0
                num_samples = 0
                sum_perf = 0
                sum_mini_steps = 0
                for item in metrics:
                    sum_loss += item.loss
                    alive_peers += 1
                    sum_perf += item.samples_per_second
                    num_samples += item.samples_accumulated
                    sum_mini_steps += item.mini_steps
                current_loss = sum_loss / max(sum_mini_steps, 1)
                logger.info(f"Epoch #{current_step}\tloss = {current_loss:.5f}")
                record = {"loss": current_loss, "alive peers": alive_peers, "samples": num_samples,
                          "performance": sum_perf, "step": latest_step}
                history.append(record)
                if wandb is not None:
                    wandb.log(record)
                if peer_args.metrics_log:
                    with open(peer_args.metrics_log, "a") as f:
                        f.write(json.dumps(record) + "\n")
                if checkpoint_handler is not None and checkpoint_handler.should_save_state(current_step):
                    checkpoint_handler.save_state(current_step)
                    if checkpoint_handler.is_time_to_upload():
                        checkpoint_handler.upload_checkpoint(current_loss)
        logger.debug("Peer is still alive...")
        if peer_args.max_iterations is None or iteration < peer_args.max_iterations:
            time.sleep(peer_args.refresh_period)
    return history


if __name__ == "__main__":
    main()
