"""Collaboration monitor of the auxiliary peer (reference ``run_aux_peer.py:21-152``).

Pieces, each usable and tested on its own:

* :func:`summarize` -- one collaboration-wide record from the per-peer ``LocalMetrics`` of an epoch:
  mean loss over every mini-step of every peer, alive peers, samples, and ``performance`` = the SUM of
  the peers' samples/s (the reference's throughput metric);
* :class:`MetricsPoller` -- reads ``{prefix}_metrics`` from the key/value store and yields a summary
  each time the newest epoch among the records advances;
* :class:`SnapshotKeeper` -- the checkpoint cadence: every ``interval`` epochs it asks the training
  group for a state snapshot (``{prefix}_state_request`` -> ``{prefix}_state``, served by rank 0's
  callback), writes ``model_state.pt`` / ``optimizer_state.pt`` in the reference's formats, and hands
  the directory to an uploader no more often than ``upload_interval`` seconds.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Callable, Iterable, List, Optional

import torch

from ..parallel.dht import get_dht_time
from .logging import get_logger

logger = get_logger(__name__)


@dataclass
class CollaborationSummary:
    step: int
    loss: float
    alive_peers: int
    samples: int
    performance: Optional[float]   # None until some peer's EMA has a measured interval

    def as_record(self) -> dict:
        """The key names the reference logs to wandb (``run_aux_peer.py:135-141``)."""
        return {"loss": self.loss, "alive peers": self.alive_peers, "samples": self.samples,
                "performance": self.performance, "step": self.step}


def summarize(records: Iterable) -> Optional[CollaborationSummary]:
    """Aggregate ``LocalMetrics``-like records (``step, loss, mini_steps, samples_accumulated,
    samples_per_second``). The loss of a peer is a SUM over its mini-steps, so the collaboration's mean
    loss divides the summed losses by the summed mini-steps."""
    records = list(records)
    if not records:
        return None
    mini = sum(int(r.mini_steps) for r in records)
    perf = sum(float(r.samples_per_second) for r in records)
    return CollaborationSummary(
        step=max(int(r.step) for r in records),
        loss=sum(float(r.loss) for r in records) / max(mini, 1),
        alive_peers=len(records),
        samples=sum(int(r.samples_accumulated) for r in records),
        # an epoch that closes before any peer's throughput EMA has an interval (epoch 0 on its first
        # micro-step) has no throughput yet: reported as None, not as 0 samples/s
        performance=perf if perf > 0 else None,
    )


class MetricsPoller:
    """``poll()`` returns a :class:`CollaborationSummary` when the collaboration reached a new epoch
    since the last call, else None. Records are parsed with ``parse`` (the schema validator)."""

    def __init__(self, dht, prefix: str, parse: Callable):
        self.dht, self.key, self.parse = dht, prefix + "_metrics", parse
        self.last_step: Optional[int] = None

    def poll(self) -> Optional[CollaborationSummary]:
        entry = self.dht.get(self.key, latest=True)
        if entry is None or not isinstance(entry.value, dict) or not entry.value:
            return None
        summary = summarize(self.parse(v.value) for v in entry.value.values())
        if summary is None or summary.step == self.last_step:
            return None
        self.last_step = summary.step
        return summary


class SnapshotKeeper:
    def __init__(self, dht, prefix: str, local_path: str, interval: Optional[int], upload_interval: Optional[float] = None,
                 uploader: Optional[Callable[[str, str], None]] = None, model: Optional[torch.nn.Module] = None,
                 fetch_timeout: float = 120.0):
        self.dht, self.prefix, self.local_path = dht, prefix, local_path
        self.interval, self.upload_interval = interval, upload_interval
        self.uploader, self.model, self.fetch_timeout = uploader, model, fetch_timeout
        self.last_saved_step = -1
        self.last_upload: Optional[float] = None
        self.epoch = 0
        os.makedirs(local_path, exist_ok=True)

    def due(self, step: int) -> bool:
        return self.interval is not None and step - self.last_saved_step >= self.interval

    def fetch(self, min_epoch: int) -> Optional[dict]:
        """Ask the training group for a snapshot of epoch >= ``min_epoch``; wait for its announcement."""
        self.dht.store(self.prefix + "_state_request", subkey=self.dht.peer_id, value=int(min_epoch),
                       expiration_time=get_dht_time() + self.fetch_timeout)
        give_up = time.time() + self.fetch_timeout
        while time.time() < give_up:
            try:
                ann = self.dht.get(self.prefix + "_state", latest=True)
            except RuntimeError:  # the store's host left
                return None
            if ann is not None and int(ann.value["epoch"]) >= min_epoch and os.path.exists(ann.value["path"]):
                return torch.load(ann.value["path"], map_location="cpu", weights_only=True)
            time.sleep(0.5)
        logger.warning(f"no training peer published a state of epoch >= {min_epoch} within {self.fetch_timeout:.0f} s")
        return None

    def save(self, step: int) -> bool:
        """Write the reference-format checkpoint files for ``step``; True if a snapshot was obtained."""
        self.last_saved_step = step
        snap = self.fetch(step)
        if snap is None:
            return False
        self.epoch = int(snap["local_epoch"])
        if self.model is not None:
            self.model.load_state_dict(snap["model"])
            model_sd = self.model.state_dict()
        else:
            model_sd = snap["model"]
        torch.save(model_sd, os.path.join(self.local_path, "model_state.pt"))
        torch.save(snap["optimizer"], os.path.join(self.local_path, "optimizer_state.pt"))
        logger.info(f"checkpoint of epoch {self.epoch} written to {self.local_path}")
        return True

    def maybe_upload(self, loss: float) -> bool:
        if self.upload_interval is None or self.uploader is None:
            return False
        now = time.time()
        if self.last_upload is not None and now - self.last_upload < self.upload_interval:
            return False
        self.last_upload = now
        try:
            self.uploader(self.local_path, f"Epoch {self.epoch}, loss {loss:.3f}")
            return True
        except Exception as e:  # noqa: BLE001 - an upload failure is logged, never fatal
            logger.warning(f"checkpoint upload failed: {e!r}")
            return False


def hub_uploader(local_path: str, repo_url: str, token: Optional[str] = None) -> Optional[Callable[[str, str], None]]:
    """A ``huggingface_hub.Repository`` push, or None when the hub library / repository is unavailable."""
    try:
        from huggingface_hub import Repository

        repo = Repository(local_dir=local_path, clone_from=repo_url, use_auth_token=token)
    except Exception as e:  # noqa: BLE001 - offline: checkpoints stay local
        logger.warning(f"Hub repository unavailable ({e!r}); checkpoints stay in {local_path}")
        return None

    def push(_path: str, message: str):
        repo.git_pull()
        repo.push_to_hub(commit_message=message)

    return push


def run_monitor(poller: MetricsPoller, keeper: Optional[SnapshotKeeper], sinks: List[Callable[[dict], None]],
                refresh_period: float, max_iterations: Optional[int] = None) -> List[dict]:
    """The aux peer's loop: poll, report each new epoch to every sink, checkpoint on cadence."""
    history = []
    it = 0
    while max_iterations is None or it < max_iterations:
        it += 1
        try:
            summary = poller.poll()
        except RuntimeError as e:  # the store's host went away: the collaboration is over
            logger.warning(f"key/value store unreachable ({e}); stopping the monitor")
            break
        if summary is not None:
            rec = summary.as_record()
            logger.info(f"epoch #{summary.step}: loss {summary.loss:.5f}, {summary.alive_peers} peers, "
                        + (f"{summary.performance:.1f} samples/s" if summary.performance is not None else "throughput n/a"))
            history.append(rec)
            for sink in sinks:
                sink(rec)
            if keeper is not None and keeper.due(summary.step) and keeper.save(summary.step):
                keeper.maybe_upload(summary.loss)
        if max_iterations is None or it < max_iterations:
            time.sleep(refresh_period)
    return history
