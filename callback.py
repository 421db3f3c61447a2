"""Trainer callback of a collaborative peer (reference ``callback.py:14-127``).

Responsibilities, each a small piece of this module:

* ``_EpochStats``   -- sums mini-step losses between optimizer epochs and turns them into one
  :class:`utils.LocalMetrics` record per epoch (published only while this peer is in sync with the
  collaboration, under its owner-signed subkey, with ``statistics_expiration``);
* NaN guard         -- one fused finiteness kernel over the parameter arena after every step; broken
  parameters roll the peer back to its last backup (or abort when it has none);
* backups           -- ``{"model", "training", "scheduler", "local_epoch"}`` at ``state_path`` every
  ``backup_every_steps`` epochs; loaded at start-up before and after ``load_state_from_peers`` (the
  second time only when newer than what the peers provided);
* ``_SnapshotServer`` -- answers auxiliary peers (which are not in the training process group): an aux
  peer posts ``{run_id}_state_request``; rank 0 writes a state snapshot to the shared filesystem and
  announces its path under ``{run_id}_state``.
"""
import os
import time
from dataclasses import dataclass

import torch
import torch.distributed as dist

from arguments import TrainingPeerArguments
from dalle_amd.ops import grads_finite
from dalle_amd.parallel.dht import get_dht_time
from dalle_amd.train.trainer import TrainerCallback
from task import TrainingTask
from utils import LocalMetrics, logger


def rank_state_path(path: str) -> str:
    """``state.zip`` for a single peer; ``state.rank{r}.zip`` for rank r of a multi-process job."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        root, ext = os.path.splitext(path)
        return f"{root}.rank{dist.get_rank()}{ext}"
    return path


@dataclass
class _EpochStats:
    loss_sum: object = 0.0  # a device scalar while the epoch runs: read once, when the epoch closes
    mini_steps: int = 0
    samples: int = 0  # samples this peer contributed to the epoch being accumulated
    contributed_total: int = 0
    reported_epoch: int = -1

    def add(self, loss):
        t = getattr(loss, "tensor", loss)  # DeferredScalar -> its tensor (no host sync per micro-step)
        self.loss_sum = self.loss_sum + (t if torch.is_tensor(t) else float(t))
        self.mini_steps += 1

    def close_epoch(self, epoch: int, samples_per_second: float) -> LocalMetrics:
        self.loss_sum = float(self.loss_sum)
        record = LocalMetrics(step=int(epoch), samples_per_second=float(samples_per_second),
                              samples_accumulated=int(self.samples), loss=float(self.loss_sum), mini_steps=int(self.mini_steps))
        self.contributed_total += self.samples
        self.reported_epoch = epoch
        self.loss_sum, self.mini_steps = 0.0, 0
        return record


class _SnapshotServer:
    def __init__(self, task: TrainingTask, share_dir: str, poll_period: float = 2.0):
        self.task, self.share_dir, self.poll_period = task, share_dir, poll_period
        self._next_poll = 0.0
        self._served = -1

    def poll(self):
        opt, dht = self.task.collaborative_optimizer, self.task.dht
        if dht is None or (dist.is_initialized() and dist.get_rank() != 0) or time.time() < self._next_poll:
            return
        self._next_poll = time.time() + self.poll_period
        request = dht.get(opt.run_id + "_state_request", latest=True)
        if request is None:
            return
        asked = request.value.values() if isinstance(request.value, dict) else [request]
        wanted = max(int(r.value) for r in asked)
        epoch = opt.local_epoch
        if wanted <= self._served or epoch < wanted:
            return
        os.makedirs(self.share_dir, exist_ok=True)
        final = os.path.abspath(os.path.join(self.share_dir, "state.pt"))
        torch.save({"model": self.task.model.state_dict(), "optimizer": opt.state_dict(),
                    "scheduler": opt.scheduler.state_dict(), "local_epoch": epoch}, final + ".tmp")
        os.replace(final + ".tmp", final)  # readers never see a half-written file
        self._served = epoch
        dht.store(opt.run_id + "_state", subkey=None, value={"path": final, "epoch": epoch},
                  expiration_time=get_dht_time() + 3600)
        logger.info(f"State snapshot of epoch {epoch} published for auxiliary peers")


class CollaborativeCallback(TrainerCallback):
    """Reports collaborative progress and reverts the peer to a backup after a numerical failure."""

    def __init__(self, task: TrainingTask, args: TrainingPeerArguments):
        super().__init__()
        self.task = task
        self.dht, self.collaborative_optimizer = task.dht, task.collaborative_optimizer
        self.statistics_expiration = args.statistics_expiration
        self.backup_every_steps = args.backup_every_steps
        self.state_path = rank_state_path(args.state_path)
        self.stats = _EpochStats()
        self._checked_version = None
        self.snapshots = _SnapshotServer(task, os.path.join(task.trainer_args.output_dir, "shared_state"))

    # -- trainer hooks ------------------------------------------------------------------------
    def on_train_begin(self, args, state, control, **kwargs):
        have_backup = os.path.isfile(self.state_path)
        if have_backup:
            self.restore_from_backup(self.state_path)
        logger.info("Synchronising with the collaboration (load_state_from_peers)")
        self.collaborative_optimizer.load_state_from_peers()
        if have_backup:  # the local backup wins only if it is at least as recent as the peers' state
            self.restore_from_backup(self.state_path, check_step=True)

    def on_step_end(self, args, state, control, **kwargs):
        control.should_log = True
        opt = self.collaborative_optimizer
        # parameters change only at global steps (a delayed update lands one local step later): check them
        # then, not after every micro-step -- the check is a device->host read
        version = (opt.local_epoch, opt.state_averager.pending)
        if version != self._checked_version and not self.params_are_finite():
            if not os.path.exists(self.state_path):
                raise RuntimeError("Parameters became NaN/Inf and there is no backup to roll back to")
            logger.warning("Parameters became NaN/Inf: rolling back to the last backup")
            self.restore_from_backup(self.state_path)
            return control
        self._checked_version = version
        if state.log_history:
            self.stats.add(state.log_history[-1]["loss"])
            if opt.local_epoch != self.stats.reported_epoch:
                self.stats.samples = getattr(opt, "last_round_samples", self.stats.samples)
                self._finish_epoch(opt)
        self.stats.samples = opt.grad_averager.local_samples_accumulated
        self.snapshots.poll()
        return control

    def _finish_epoch(self, opt):
        sps = opt.tracker.performance_ema.samples_per_second
        steps, loss = self.stats.mini_steps, self.stats.loss_sum
        record = self.stats.close_epoch(opt.local_epoch, sps)
        logger.info(f"epoch {opt.local_epoch}: contributed {self.stats.contributed_total} samples so far, "
                    f"{sps:.2f} samples/s" + (f", mean loss {loss / steps:.5f}" if steps else ""))
        in_sync = opt.local_epoch == opt.tracker.global_epoch
        if self.dht is not None and in_sync:
            payload = record.model_dump() if hasattr(record, "model_dump") else record.dict()
            self.dht.store(key=opt.run_id + "_metrics", subkey=self.task.local_public_key, value=payload,
                           expiration_time=get_dht_time() + self.statistics_expiration, return_future=True)
        if self.backup_every_steps is not None and opt.local_epoch % self.backup_every_steps == 0:
            self.backup_state()

    # -- numerics / backups ---------------------------------------------------------------------
    @torch.no_grad()
    def params_are_finite(self) -> bool:
        arena = getattr(self.task, "_arena", None)
        if arena is not None:  # one fused kernel over every parameter
            return grads_finite(arena.data)
        return all(bool(torch.isfinite(p).all()) for p in self.task.model.parameters())

    @torch.no_grad()
    def backup_state(self):
        opt = self.collaborative_optimizer
        logger.info(f"Writing backup of epoch {opt.local_epoch} to {self.state_path}")
        snapshot = {"model": self.task.model.state_dict(), "training": opt.state_dict(),
                    "scheduler": opt.state_averager.scheduler.state_dict(), "local_epoch": opt.local_epoch}
        # every peer owns its file (ranks of one node must not write the same path) and a reader never
        # sees a torn file: write a temporary, then rename it into place
        torch.save(snapshot, self.state_path + ".tmp")
        os.replace(self.state_path + ".tmp", self.state_path)

    @torch.no_grad()
    def restore_from_backup(self, path, check_step: bool = False):
        snapshot = torch.load(path, map_location="cpu", weights_only=True)
        opt = self.collaborative_optimizer
        if check_step and snapshot["local_epoch"] < opt.local_epoch:
            logger.info(f"Backup (epoch {snapshot['local_epoch']}) is older than the current state "
                        f"(epoch {opt.local_epoch}); keeping the current state")
            return
        self.task.model.load_state_dict(snapshot["model"], strict=True)  # our own backup: every key must match
        opt.load_state_dict(snapshot["training"])
        opt.state_averager.scheduler.load_state_dict(snapshot["scheduler"])
        opt.state_averager.local_epoch = snapshot["local_epoch"]
        logger.info(f"Restored the backup of epoch {snapshot['local_epoch']}")
