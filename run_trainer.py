#!/usr/bin/env python3
"""Training peer entrypoint (reference ``run_trainer.py:1-60``), CLI-compatible.

One peer per MI355X: launch with ``torchrun --nproc-per-node 8 --master-addr 127.0.0.1 run_trainer.py ...``
(RCCL over xGMI between the 8 peers of a node), or a single process for one GPU / CPU.
"""
import os
from pathlib import Path

import torch

import callback
import utils
from arguments import CollaborativeArguments, HFTrainerArguments, TrainingPeerArguments
from dalle_amd.train.trainer import CollaborativeHFTrainer, PrinterCallback, ProgressCallback
from dalle_amd.utils.argparse import HfArgumentParser
from dalle_amd.utils.logging import get_logger, use_hivemind_log_handler
from task import TrainingTask

use_hivemind_log_handler("in_root_logger")
logger = get_logger(__name__)

torch.set_num_threads(int(os.environ.get("DALLE_AMD_CPU_THREADS", "1")))  # Otherwise, it becomes very slow on machines with ~100 CPUs


def main(argv=None):
    parser = HfArgumentParser((TrainingPeerArguments, HFTrainerArguments, CollaborativeArguments))
    training_peer_args, trainer_args, collab_args = parser.parse_args_into_dataclasses(argv)
    if trainer_args.local_rank < 0 and "LOCAL_RANK" in os.environ:
        trainer_args.local_rank = int(os.environ["LOCAL_RANK"])

    logger.info(f"Trying {len(training_peer_args.initial_peers)} initial peers: {training_peer_args.initial_peers}")

    utils.log_process_rank(trainer_args)
    task = TrainingTask(training_peer_args, trainer_args, collab_args)
    model = task.model.to(trainer_args.device)

    collaborative_callback = callback.CollaborativeCallback(task, training_peer_args)
    assert trainer_args.do_train and not trainer_args.do_eval

    trainer = CollaborativeHFTrainer(
        model=model,
        args=trainer_args,
        tokenizer=task.tokenizer,
        data_collator=task.data_collator,
        data_seed=int.from_bytes(task.local_public_key[-8:], "little"),
        train_dataset=task.training_dataset,
        eval_dataset=None,
        collaborative_optimizer=task.collaborative_optimizer,
        callbacks=[collaborative_callback],
    )
    trainer.remove_callback(PrinterCallback)
    trainer.remove_callback(ProgressCallback)

    latest_checkpoint_dir = max(Path(trainer_args.output_dir).glob("checkpoint*"), key=os.path.getctime, default=None)
    trainer.train(model_path=latest_checkpoint_dir)
    return trainer, task


if __name__ == "__main__":
    main()
