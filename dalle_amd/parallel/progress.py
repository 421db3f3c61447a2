"""Training-progress tracking across peers (``callback.py:63,79``).

Each peer reports ``(epoch, samples_accumulated, samples_per_second)``; the collaboration's global
epoch advances when the peers of the current epoch together accumulated ``target_batch_size``
samples.

Transports:
* ``store`` (default for the ranks of a torch.distributed group -- one process per MI355X, RCCL over
  xGMI): asynchronous progress records, no collective and no device sync per micro-step. Every peer
  adds the samples it just accumulated to ONE atomic counter per epoch in the job's c10d key/value
  store (``store.add``: one small TCP round trip, the reply is the collaboration-wide total). Peers
  run at their own pace -- a faster GPU contributes more samples -- and each one enters the epoch's
  averaging round as soon as the total it sees reaches ``target_batch_size`` (all peers see the same
  monotone counter, so they arrive within one local step of each other). The exact per-peer sample
  counts are exchanged by ONE tiny all-gather at the round itself (``CollaborativeOptimizer``).
* ``static``: homogeneous peers with a fixed batch each step -- the global count is ``local * world``;
  no communication at all (the headline benchmark).
* ``collective``: one tiny all-reduce per local step (lockstep; kept for the elastic generations,
  whose per-generation stores are short-lived).
* ``dht`` (loosely coupled peers, e.g. the auxiliary monitor): records under ``{prefix}_progress``
  in the native key/value store, fetched periodically.
* ``local``: a single peer.

In every mode the local record is also published to the key/value store (if any) for monitoring.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, asdict
from typing import Optional

import torch
import torch.distributed as dist

from .dht import get_dht_time
from ..utils.logging import get_logger

logger = get_logger(__name__)


@dataclass
class LocalTrainingProgress:
    peer_id: str
    epoch: int
    samples_accumulated: int
    samples_per_second: float
    time: float
    client_mode: bool


@dataclass
class GlobalTrainingProgress:
    epoch: int
    samples_accumulated: int
    target_batch_size: int
    num_peers: int
    num_clients: int
    eta_next_epoch: float
    next_fetch_time: float


class PerformanceEMA:
    """Exponential moving average of samples/s (``tracker.performance_ema``; the reference's throughput
    metric, ``callback.py:63``, summed over peers by the aux peer, ``run_aux_peer.py:129,141``).

    On a GPU peer the intervals are DEVICE time: every ``update`` records an event on the current stream
    and an interval is the time between two consecutive events' completions on the device, read once the
    later event has completed (non-blocking; the value lags the host by the queue depth). Host
    ``perf_counter`` deltas between calls would measure how fast the host ENQUEUES work -- with no
    per-step device sync they run ahead of the GPU (the warm-up queue fill biased the round-2 value up
    to +11 % over wall clock). The first ``warmup`` intervals are dropped. On CPU peers the host clock is
    the device clock."""

    def __init__(self, alpha: float = 0.1, eps: float = 1e-20, device=None, warmup: int = 2):
        self.alpha, self.eps = alpha, eps
        self.ema_seconds_per_sample = 0.0
        self._sps = 0.0
        self.num_updates = 0
        self.timestamp = time.perf_counter()
        self.paused = False
        self.warmup = int(warmup)
        self._seen = 0  # intervals observed (including the dropped warm-up ones)
        dev = torch.device(device) if device is not None else None
        self._events = dev is not None and dev.type == "cuda" and torch.cuda.is_available()
        self._device = dev
        self._pending = []   # (event, task_size, counted) in record order
        self._last_event = None

    def _record(self):
        """An event on the current device stream (query / elapsed_time / synchronize)."""
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self._device))
        return ev

    def _ema(self, task_size: float, interval: float):
        self._seen += 1
        if self._seen <= self.warmup:
            return
        self.num_updates += 1
        adjusted = self.alpha / (1 - (1 - self.alpha) ** self.num_updates)
        self.ema_seconds_per_sample = adjusted * interval / task_size + (1 - adjusted) * self.ema_seconds_per_sample
        self._sps = 1.0 / max(self.ema_seconds_per_sample, self.eps)

    def _drain(self):
        while self._pending and self._pending[0][0].query():
            ev, task_size, counted = self._pending.pop(0)
            if self._last_event is not None and counted and task_size > 0:
                self._ema(task_size, self._last_event.elapsed_time(ev) / 1e3)
            self._last_event = ev

    @property
    def samples_per_second(self) -> float:
        if self._events:
            self._drain()
        return self._sps

    @samples_per_second.setter
    def samples_per_second(self, v: float):
        self._sps = float(v)

    def update(self, task_size: float, interval: Optional[float] = None) -> float:
        if self._events and interval is None:
            self._pending.append((self._record(), float(task_size), not self.paused))
            self._drain()
            return self._sps
        now = time.perf_counter()
        if interval is None:
            interval = now - self.timestamp
        self.timestamp = now
        if task_size <= 0 or self.paused:
            return self._sps
        self._ema(task_size, interval)
        return self._sps

    def flush(self) -> float:
        """Wait for every recorded event and fold in its interval (end of a measurement)."""
        if self._events:
            for ev, _, _ in self._pending:
                ev.synchronize()
            self._drain()
        return self._sps

    def reset_timer(self):
        self.timestamp = time.perf_counter()
        self._last_event = None
        self._pending = [(ev, t, False) for ev, t, _ in self._pending]

    def pause(self):
        self.paused = True

    def resume(self):
        self.paused = False
        self.reset_timer()


class ProgressTracker:
    def __init__(self, dht=None, prefix: str = "run", target_batch_size: int = 4096, group=None, device=None,
                 client_mode: bool = False, peer_id: str = "local", mode: str = "collective",
                 metadata_expiration: float = 60.0, report_period: float = 1.0, performance_ema_alpha: float = 0.1,
                 max_wait_time: Optional[float] = None, store=None):
        self.dht, self.prefix = dht, prefix
        self.target_batch_size = target_batch_size
        self.group = group
        self.device = device if device is not None else torch.device("cpu")
        self.client_mode = client_mode
        self.peer_id = peer_id
        grouped = dist.is_available() and dist.is_initialized()
        if mode in ("collective", "store", "static") and not grouped:
            mode = "local"
        self.mode = mode
        self.store = None
        if mode == "store":
            # the job's store (torchrun: hosted by the elastic agent), or an explicit long-lived one
            self.store = store if store is not None else dist.distributed_c10d._get_default_store()
            self._ns = f"collab/{prefix}"
            self._reported = 0  # samples of the current epoch already added to the shared counter
        self.metadata_expiration = metadata_expiration
        self.report_period = report_period
        self.max_wait_time = max_wait_time
        self.performance_ema = PerformanceEMA(alpha=performance_ema_alpha, device=self.device)
        self.local_progress = LocalTrainingProgress(peer_id, 0, 0, 0.0, get_dht_time(), client_mode)
        self.global_progress = GlobalTrainingProgress(0, 0, target_batch_size, 1, int(client_mode), float("inf"), 0.0)
        self.max_epoch_seen = 0
        self.min_epoch_seen = None  # "collective" mode: the lowest epoch of any peer at the last update
        self._last_report = 0.0
        self._epoch_start = time.perf_counter()
        self._publish_lock = threading.Lock()

    @property
    def progress_key(self) -> str:
        return f"{self.prefix}_progress"

    @property
    def global_epoch(self) -> int:
        return self.global_progress.epoch

    # ------------------------------------------------------------------------------------------
    def report_local_progress(self, local_epoch: int, samples_accumulated: int, update_global_samples: bool = True):
        prev = self.local_progress.samples_accumulated if self.local_progress.epoch == local_epoch else 0
        self.performance_ema.update(task_size=max(0, samples_accumulated - prev))
        self.local_progress = LocalTrainingProgress(self.peer_id, local_epoch, samples_accumulated,
                                                    self.performance_ema.samples_per_second, get_dht_time(),
                                                    self.client_mode)
        if self.mode == "store":
            self._store_update(local_epoch, samples_accumulated)
        elif self.mode == "collective":
            self._collective_update()
        elif self.mode == "static":
            # every rank contributes the same batch per step (asserted by the caller): the global count
            # is known without a collective, so no per-step host sync
            world = dist.get_world_size(self.group) if dist.is_initialized() else 1
            total = samples_accumulated * world
            self.global_progress = GlobalTrainingProgress(local_epoch, total, self.target_batch_size, world, 0,
                                                          self._eta(total), 0.0)
            self.max_epoch_seen = max(self.max_epoch_seen, local_epoch)
        elif self.mode == "local":
            self.global_progress = GlobalTrainingProgress(local_epoch, samples_accumulated, self.target_batch_size, 1,
                                                          int(self.client_mode), self._eta(samples_accumulated), 0.0)
            self.max_epoch_seen = max(self.max_epoch_seen, local_epoch)
        else:
            self._dht_update()
        self._maybe_publish()

    def _eta(self, samples: int) -> float:
        sps = self.performance_ema.samples_per_second * max(1, self.global_progress.num_peers)
        remaining = max(0, self.target_batch_size - samples)
        return get_dht_time() + (remaining / sps if sps > 0 else float("inf"))

    def _store_update(self, local_epoch: int, samples_accumulated: int):
        delta = max(0, int(samples_accumulated) - self._reported)
        if self.max_wait_time is not None and time.perf_counter() - self._epoch_start > self.max_wait_time \
                and samples_accumulated > 0:
            delta += self.target_batch_size  # ETA deadline: close the epoch for everyone (the round counts exactly)
        total = int(self.store.add(f"{self._ns}/e{local_epoch}/samples", delta))
        self._reported = int(samples_accumulated)
        world = dist.get_world_size(self.group) if dist.is_initialized() else 1
        self.max_epoch_seen = max(self.max_epoch_seen, local_epoch)
        self.global_progress = GlobalTrainingProgress(local_epoch, total, self.target_batch_size, world,
                                                      int(self.client_mode), self._eta(total), 0.0)

    def _collective_update(self):
        lp = self.local_progress
        dt = torch.float64 if self.device.type == "cpu" else torch.float32
        s = torch.tensor([lp.samples_accumulated, lp.samples_per_second, 1.0, float(lp.client_mode)], dtype=dt, device=self.device)
        e = torch.tensor([float(lp.epoch), -float(lp.epoch)], dtype=dt, device=self.device)
        dist.all_reduce(s, group=self.group)
        dist.all_reduce(e, op=dist.ReduceOp.MAX, group=self.group)  # (max epoch, -min epoch)
        s = s.tolist()
        e = e.tolist()
        max_epoch = int(e[0])
        self.max_epoch_seen = max_epoch
        self.min_epoch_seen = int(-e[1])
        total, sps, peers, clients = int(round(s[0])), s[1], int(round(s[2])), int(round(s[3]))
        remaining = max(0, self.target_batch_size - total)
        eta = get_dht_time() + (remaining / sps if sps > 0 else float("inf"))
        self.global_progress = GlobalTrainingProgress(max_epoch, total, self.target_batch_size, peers, clients, eta, 0.0)

    def _dht_update(self):
        if self.dht is None:
            return
        now = get_dht_time()
        if now < self.global_progress.next_fetch_time:
            return
        self._publish(force=True)
        entry = self.dht.get(self.progress_key, latest=True)
        peers = []
        if entry is not None and isinstance(entry.value, dict):
            for v in entry.value.values():
                try:
                    peers.append(LocalTrainingProgress(**v.value))
                except TypeError:
                    continue
        if not peers:
            peers = [self.local_progress]
        epoch = max(p.epoch for p in peers)
        cur = [p for p in peers if p.epoch == epoch]
        total = sum(p.samples_accumulated for p in cur)
        sps = sum(p.samples_per_second for p in cur)
        remaining = max(0, self.target_batch_size - total)
        eta = now + (remaining / sps if sps > 0 else float("inf"))
        self.max_epoch_seen = epoch
        self.global_progress = GlobalTrainingProgress(epoch, total, self.target_batch_size, len(peers),
                                                      sum(p.client_mode for p in peers), eta,
                                                      now + min(self.report_period, max(0.1, eta - now)))

    def _publish(self, force: bool = False):
        if self.dht is None:
            return
        now = get_dht_time()
        if not force and now - self._last_report < self.report_period:
            return
        self._last_report = now
        try:
            self.dht.store(self.progress_key, subkey=self.peer_id, value=asdict(self.local_progress),
                           expiration_time=now + self.metadata_expiration, return_future=True)
        except Exception as e:  # monitoring must never break training
            logger.debug(f"progress publish failed: {e}")

    def _maybe_publish(self):
        self._publish(force=False)

    # ------------------------------------------------------------------------------------------
    @property
    def ready_to_update_epoch(self) -> bool:
        gp = self.global_progress
        if gp.samples_accumulated >= self.target_batch_size:
            return True
        if self.max_wait_time is not None and time.perf_counter() - self._epoch_start > self.max_wait_time and gp.samples_accumulated > 0:
            return True
        return False

    def update_epoch(self, new_epoch: int):
        if self.mode == "store":
            self._reported = 0
        self.local_progress = LocalTrainingProgress(self.peer_id, new_epoch, 0, self.performance_ema.samples_per_second,
                                                    get_dht_time(), self.client_mode)
        self.global_progress = GlobalTrainingProgress(max(new_epoch, self.global_progress.epoch), 0, self.target_batch_size,
                                                      self.global_progress.num_peers, self.global_progress.num_clients,
                                                      float("inf"), 0.0)
        self._epoch_start = time.perf_counter()
        self._publish(force=True)

    def shutdown(self):
        pass
