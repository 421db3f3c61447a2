#!/usr/bin/env python3
"""Training peer (counterpart of the reference ``run_trainer.py``; same flags).

A peer is one process driving one MI355X. On a node:
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 run_trainer.py <flags>
gives 8 peers whose gradients average over RCCL / xGMI; a single process trains on one GPU (or the
CPU). The trainer resumes from the newest ``<output_dir>/checkpoint*`` when there is one.
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

# host threads stay few: the GPU does the work, and ~100-core hosts otherwise oversubscribe
torch.set_num_threads(int(os.environ.get("DALLE_AMD_CPU_THREADS", "1")))


def _newest_checkpoint(output_dir: str):
    candidates = list(Path(output_dir).glob("checkpoint*"))
    return max(candidates, key=os.path.getctime) if candidates else None


def main(argv=None):
    peer_args, trainer_args, collab_args = HfArgumentParser(
        (TrainingPeerArguments, HFTrainerArguments, CollaborativeArguments)).parse_cli_or_file(argv)
    if trainer_args.local_rank < 0 and "LOCAL_RANK" in os.environ:  # torchrun
        trainer_args.local_rank = int(os.environ["LOCAL_RANK"])
    if not trainer_args.do_train or trainer_args.do_eval:
        raise ValueError("a training peer runs with --do_train True --do_eval False")
    if torch.cuda.is_available() and trainer_args.per_device_train_batch_size < 16:
        # the reference's default (2) is sized for 16 GB T4s: on MI355X it gives GEMMs of M = 2,560 tokens,
        # launch-bound; 48 was the measured optimum of the bench sweep (README "Running")
        logger.warning(f"per_device_train_batch_size={trainer_args.per_device_train_batch_size} leaves an MI355X mostly "
                       f"idle; --per_device_train_batch_size 48 is the measured optimum (72 GB of HBM)")
    logger.info(f"initial peers ({len(peer_args.initial_peers)}): {peer_args.initial_peers}")
    utils.log_process_rank(trainer_args)

    task = TrainingTask(peer_args, trainer_args, collab_args)
    trainer = CollaborativeHFTrainer(
        model=task.model.to(trainer_args.device),
        args=trainer_args,
        tokenizer=task.tokenizer,
        data_collator=task.data_collator,
        # a stable per-peer data order (the reference's hash() of bytes is salted per process)
        data_seed=int.from_bytes(task.local_public_key[-8:], "little"),
        train_dataset=task.training_dataset,
        eval_dataset=None,
        collaborative_optimizer=task.collaborative_optimizer,
        callbacks=[callback.CollaborativeCallback(task, peer_args)],
    )
    # progress is reported by the collaborative callback (per epoch, across peers), not per mini-step
    for cb in (PrinterCallback, ProgressCallback):
        trainer.remove_callback(cb)
    trainer.train(model_path=_newest_checkpoint(trainer_args.output_dir))
    return trainer, task


def _teardown(task) -> None:
    """Release the communicator before the interpreter exits: a gloo / RCCL group still alive at interpreter
    finalisation tears its worker threads down in arbitrary order (an occasional SIGABRT after a finished
    run). Local only -- the key/value store host stays up for peers still writing their last records."""
    import torch.distributed as dist

    try:
        if getattr(task, "_elastic", None) is not None:
            task._elastic.shutdown()
        elif dist.is_available() and dist.is_initialized():
            dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 - teardown of a broken group must not fail a finished run
        logger.warning(f"process group teardown: {e!r}")


if __name__ == "__main__":
    _trainer, _task = main()
    _teardown(_task)
