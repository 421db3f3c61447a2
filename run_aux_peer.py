#!/usr/bin/env python3
"""Auxiliary peer: collaboration monitor + checkpointer (reference ``run_aux_peer.py``).

Joins the key/value store, and every ``refresh_period`` seconds turns the peers' ``{prefix}_metrics``
records into one collaboration summary (``dalle_amd.utils.monitor``: mean loss, alive peers, samples,
throughput = sum of the peers' samples/s), logged to wandb when installed and/or a JSON-lines file.
Every ``save_checkpoint_step_interval`` epochs it fetches a state snapshot from the training group and
writes ``model_state.pt`` / ``optimizer_state.pt``; with ``repo_url`` + ``upload_interval`` those are
pushed to the Hub (when ``huggingface_hub`` can reach it). The aux peer may also host the coordinator
store that elastic trainers rendezvous on.
"""
import json

import utils
from arguments import AuxiliaryPeerArguments, CollaborativeArguments, HFTrainerArguments
from dalle_amd.utils.argparse import HfArgumentParser
from dalle_amd.utils.logging import get_logger, use_hivemind_log_handler
from dalle_amd.utils.monitor import MetricsPoller, SnapshotKeeper, hub_uploader, run_monitor
from task import TrainingTask

use_hivemind_log_handler("in_root_logger")
logger = get_logger(__name__)


def _sinks(peer_args):
    sinks = []
    if peer_args.wandb_project is not None:
        try:
            import wandb

            wandb.init(project=peer_args.wandb_project)
            sinks.append(wandb.log)
        except ImportError:
            logger.warning("wandb is not installed; use --metrics_log for a local JSON-lines log")
    if peer_args.metrics_log:
        path = peer_args.metrics_log

        def to_file(rec):
            with open(path, "a") as f:
                f.write(json.dumps(rec) + "\n")
        sinks.append(to_file)
    return sinks


def main(argv=None):
    parser = HfArgumentParser((AuxiliaryPeerArguments, HFTrainerArguments, CollaborativeArguments))
    peer_args, trainer_args, collab_args = parser.parse_cli_or_file(argv)
    if peer_args.assist_in_averaging:
        raise NotImplementedError("aux peers are not members of the RCCL averaging group (as in the reference)")

    if peer_args.host_elastic_coordinator and peer_args.elastic_coordinator:
        # the store elastic trainers rendezvous on must outlive every trainer
        from dalle_amd.parallel.elastic import coordinator_store

        host, port = peer_args.elastic_coordinator.rsplit(":", 1)
        _coordinator = coordinator_store(host, int(port), is_master=True)  # noqa: F841 - kept alive by this frame
        logger.info(f"elastic coordinator store at {peer_args.elastic_coordinator}")
        peer_args.elastic_coordinator = None  # this process is not a trainer / group member

    task = TrainingTask(peer_args, trainer_args, collab_args)
    dht = task.dht
    keeper = None
    if peer_args.store_checkpoints:
        uploader = None
        if peer_args.upload_interval is not None and peer_args.repo_url:
            uploader = hub_uploader(peer_args.local_path, peer_args.repo_url,
                                    getattr(task.authorizer, "hf_user_access_token", None))
        keeper = SnapshotKeeper(dht, peer_args.experiment_prefix, peer_args.local_path,
                                peer_args.save_checkpoint_step_interval, peer_args.upload_interval, uploader,
                                model=task.model)
    poller = MetricsPoller(dht, peer_args.experiment_prefix, utils.LocalMetrics.model_validate)
    return run_monitor(poller, keeper, _sinks(peer_args), peer_args.refresh_period, peer_args.max_iterations)


if __name__ == "__main__":
    main()
