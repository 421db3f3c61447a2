"""CollaborativeCallback: progress reporting, NaN rollback and backups (reference ``callback.py:14-127``).

Also serves state snapshots to auxiliary peers (which are not members of the training process
group): an aux peer posts ``{run_id}_state_request``; the group's rank 0 answers with a
``torch.save`` snapshot on the shared filesystem announced under ``{run_id}_state``.
"""
import os.path
import time
from typing import Any

import torch
import torch.distributed as dist

from arguments import TrainingPeerArguments
from dalle_amd.ops import grads_finite
from dalle_amd.parallel.dht import get_dht_time
from dalle_amd.train.trainer import TrainerCallback
from task import TrainingTask
from utils import LocalMetrics, logger


class CollaborativeCallback(TrainerCallback):
    """
    This callback monitors and reports collaborative training progress,
    In case of a catastrophic failure, it can also revert training to a backup
    """

    def __init__(self, task: TrainingTask, args: TrainingPeerArguments):
        super().__init__()
        self.task = task
        self.dht, self.collaborative_optimizer = task.dht, task.collaborative_optimizer
        self.statistics_expiration = args.statistics_expiration
        self.last_reported_collaboration_step = -1
        self.samples = 0
        self.steps = 0
        self.loss = 0
        self.total_samples_processed = 0
        self.backup_every_steps = args.backup_every_steps
        self.state_path = args.state_path
        self.share_dir = os.path.join(task.trainer_args.output_dir, "shared_state")
        self._last_request_check = 0.0
        self._served_epoch = -1

    def on_train_begin(self, args, state, control, **kwargs):
        if os.path.isfile(self.state_path):
            self.restore_from_backup(self.state_path)
            logger.info("Loaded state")

        logger.info("Loading state from peers")
        self.collaborative_optimizer.load_state_from_peers()

        if os.path.isfile(self.state_path):
            self.restore_from_backup(self.state_path, check_step=True)

    def on_step_end(self, args, state, control, **kwargs):
        control.should_log = True
        if not self.params_are_finite():
            if not os.path.exists(self.state_path):
                raise RuntimeError("Encountered broken parameters, but there is no backup to fall back to.")
            logger.warning("Parameters are invalid, reloading model from earlier state")
            self.restore_from_backup(self.state_path)
            return control

        if state.log_history:
            self.loss += state.log_history[-1]["loss"]
            self.steps += 1
            if self.collaborative_optimizer.local_epoch != self.last_reported_collaboration_step:
                self.last_reported_collaboration_step = self.collaborative_optimizer.local_epoch
                self.total_samples_processed += self.samples
                samples_per_second = self.collaborative_optimizer.tracker.performance_ema.samples_per_second
                statistics = LocalMetrics(
                    step=self.collaborative_optimizer.local_epoch,
                    samples_per_second=float(samples_per_second),
                    samples_accumulated=self.samples,
                    loss=float(self.loss),
                    mini_steps=self.steps,
                )
                logger.info(f"Current epoch: {self.collaborative_optimizer.local_epoch}")
                logger.info(f"Your current contribution: {self.total_samples_processed} samples")
                logger.info(f"Performance: {samples_per_second} samples/sec")
                if self.steps:
                    logger.info(f"Local loss: {self.loss / self.steps}")

                self.loss = 0
                self.steps = 0
                if self.dht is not None and self.collaborative_optimizer.local_epoch == self.collaborative_optimizer.tracker.global_epoch:
                    self.dht.store(
                        key=self.collaborative_optimizer.run_id + "_metrics",
                        subkey=self.task.local_public_key,
                        value=statistics.model_dump() if hasattr(statistics, "model_dump") else statistics.dict(),
                        expiration_time=get_dht_time() + self.statistics_expiration,
                        return_future=True,
                    )
                if self.backup_every_steps is not None and \
                        self.collaborative_optimizer.local_epoch % self.backup_every_steps == 0:
                    self.backup_state()

        self.samples = self.collaborative_optimizer.grad_averager.local_samples_accumulated
        self.serve_state_requests()
        return control

    @torch.no_grad()
    def params_are_finite(self):
        arena = getattr(self.task, "_arena", None)
        if arena is not None:
            return grads_finite(arena.data)
        for param in self.task.model.parameters():
            if not torch.all(torch.isfinite(param)):
                return False
        return True

    @torch.no_grad()
    def backup_state(self) -> Any:
        logger.info("Saving backup")
        return torch.save(
            {
                "model": self.task.model.state_dict(),
                "training": self.collaborative_optimizer.state_dict(),
                "scheduler": self.collaborative_optimizer.state_averager.scheduler.state_dict(),
                "local_epoch": self.collaborative_optimizer.local_epoch,
            },
            self.state_path,
        )

    @torch.no_grad()
    def restore_from_backup(self, path, check_step=False):
        state = torch.load(path, map_location="cpu", weights_only=True)
        current_step = self.collaborative_optimizer.local_epoch
        backup_step = state['local_epoch']
        if not check_step or backup_step >= current_step:
            self.task.model.load_state_dict(state["model"], strict=False)
            self.collaborative_optimizer.load_state_dict(state["training"])
            self.collaborative_optimizer.state_averager.scheduler.load_state_dict(state["scheduler"])
            self.collaborative_optimizer.state_averager.local_epoch = backup_step
            logger.info("Restored from a backup")
        else:
            logger.info("Bypassed restoring state from local backup: backup state is too old.")

    # -- state snapshots for auxiliary peers ------------------------------------------------------
    def serve_state_requests(self, min_period: float = 2.0):
        if self.dht is None or (dist.is_initialized() and dist.get_rank() != 0):
            return
        now = time.time()
        if now - self._last_request_check < min_period:
            return
        self._last_request_check = now
        run_id = self.collaborative_optimizer.run_id
        req = self.dht.get(run_id + "_state_request", latest=True)
        if req is None:
            return
        wanted = max([int(v.value) for v in req.value.values()] if isinstance(req.value, dict) else [int(req.value)])
        epoch = self.collaborative_optimizer.local_epoch
        if wanted <= self._served_epoch or epoch < wanted:
            return
        os.makedirs(self.share_dir, exist_ok=True)
        path = os.path.abspath(os.path.join(self.share_dir, "state.pt"))
        tmp = path + ".tmp"
        torch.save({"model": self.task.model.state_dict(), "optimizer": self.collaborative_optimizer.state_dict(),
                    "scheduler": self.collaborative_optimizer.scheduler.state_dict(), "local_epoch": epoch}, tmp)
        os.replace(tmp, path)
        self._served_epoch = epoch
        self.dht.store(run_id + "_state", subkey=None, value={"path": path, "epoch": epoch}, expiration_time=get_dht_time() + 3600)
        logger.info(f"served a state snapshot of epoch {epoch} to auxiliary peers")
