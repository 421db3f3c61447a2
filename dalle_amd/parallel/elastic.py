"""Elastic membership for the collaborative optimizer ("new build").

hivemind peers come and go at any time; a torch.distributed (RCCL/gloo) communicator cannot survive a
member's death. This module gives the process group a LIFECYCLE driven by a coordinator store that
outlives any single trainer (a ``torch.distributed.TCPStore`` served by the aux peer / launcher, or
any process that is not itself a trainer):

* **generations** -- every communicator belongs to generation ``g``. Peers joining generation ``g``
  take an arrival ticket (atomic ``add``); the first arrival is the leader and freezes the member list
  after ``matchmaking_time`` seconds (or as soon as ``min_peers`` arrived... whichever is later within
  the window). Ranks are ticket order; the group is built over a ``PrefixStore("g{g}")`` of the shared
  store, so generations never see each other's keys.
* **failure** -- collectives run under a timeout (the watchdog: ``allreduce_timeout``); a dead peer makes
  them raise (gloo: connection closed; RCCL: ``Work.wait`` timeout). The survivors then ``regroup()``:
  abort the old communicator (never a blocking teardown) and rendezvous in generation ``g + 1``. Whoever arrives first
  bumps the generation counter with a compare-and-set, so a failure seen by several ranks bumps it once.
* **joining** -- a peer that arrives after a generation froze raises the ``join_pending`` flag and waits
  for the next generation; members poll the flag once per global step (``poll_join``: one store read
  plus one 1-element MAX all-reduce so every member decides identically) and regroup together. The
  joiner then receives parameters / optimizer state from a donor (``load_state_from_peers``).
"""
from __future__ import annotations

import datetime
import os
import threading
import time
from typing import List, Optional

import torch
import torch.distributed as dist

from ..utils.logging import get_logger
from .watchdog import abort_group

logger = get_logger(__name__)


def coordinator_store(host: str, port: int, is_master: bool, timeout: float = 300.0) -> dist.TCPStore:
    """The long-lived store the generations rendezvous on (``is_master`` on the coordinator process)."""
    return dist.TCPStore(host, port, world_size=None, is_master=is_master, timeout=datetime.timedelta(seconds=timeout),
                         wait_for_workers=False)


def recovery_store(run_id: str, timeout: float = 300.0) -> Optional[dist.Store]:
    """A key/value store that OUTLIVES every trainer process, for re-forming the group after a failure on
    the default launch path, or None:

    * ``DALLE_AMD_COORDINATOR=host:port`` -- an external coordinator (aux peer, launcher, test harness);
    * a torchrun worker (``TORCHELASTIC_USE_AGENT_STORE=True``): the elastic AGENT hosts the job's
      TCPStore at ``MASTER_ADDR:MASTER_PORT`` -- not the rank-0 worker -- so it survives any worker.

    Keys live under ``dalle_recovery/{run_id}``, and under a per-attempt suffix when torchrun restarts the
    workers (``--max-restarts``: TORCHELASTIC_RESTART_COUNT > 0): the agent's store keeps the previous
    attempt's generations, which must not leak into the fresh world (it resumes from its checkpoint)."""
    spec = os.environ.get("DALLE_AMD_COORDINATOR")
    try:
        if spec:
            host, port = spec.rsplit(":", 1)
            base = coordinator_store(host, int(port), is_master=False, timeout=timeout)
        elif os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true" and "MASTER_PORT" in os.environ:
            base = coordinator_store(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]), is_master=False,
                                     timeout=timeout)
        else:
            return None
    except Exception as e:  # noqa: BLE001 - no recovery store: the caller falls back to detaching
        logger.warning(f"[elastic] recovery store unavailable ({e!r})")
        return None
    attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") if not spec else "0"
    return dist.PrefixStore(f"dalle_recovery/{run_id}" + (f"/attempt{attempt}" if attempt not in ("", "0") else ""), base)


class ElasticGroup:
    def __init__(self, store: dist.Store, peer_id: str, backend: str = "gloo", matchmaking_time: float = 5.0,
                 allreduce_timeout: float = 60.0, min_peers: int = 1, device: Optional[torch.device] = None,
                 heartbeat_interval: float = 0.5, heartbeat_timeout: float = 3.0):
        self.store = store
        self.peer_id = str(peer_id)
        self.backend = backend
        self.matchmaking_time = float(matchmaking_time)
        self.timeout = float(allreduce_timeout)
        self.min_peers = int(min_peers)
        self.device = device or torch.device("cpu")
        self.generation = -1
        self.members: List[str] = []
        self.rank, self.world_size = -1, 0
        self.regroups = 0
        # liveness: a heartbeat key per peer, so a regroup leader can tell a slow survivor (fresh heartbeat:
        # wait for it) from a dead member (stale heartbeat: go on without it)
        self.hb_interval, self.hb_timeout = float(heartbeat_interval), float(heartbeat_timeout)
        self._hb_stop = threading.Event()
        self._hb = threading.Thread(target=self._heartbeat, daemon=True)
        self._hb.start()

    def _heartbeat(self):
        while not self._hb_stop.is_set():
            try:
                self.store.set(f"elastic/hb/{self.peer_id}", repr(time.time()))
            except Exception:  # noqa: BLE001 - the coordinator may be gone at shutdown
                return
            self._hb_stop.wait(self.hb_interval)

    def _alive(self, peer: str) -> bool:
        try:
            return time.time() - float(self.store.get(f"elastic/hb/{peer}")) < self.hb_timeout
        except Exception:  # noqa: BLE001
            return False

    @classmethod
    def adopt(cls, store: dist.Store, rank: int, world_size: int, backend: str, **kw) -> "ElasticGroup":
        """Take over an EXISTING process group (the torchrun world) as generation -1: no rendezvous now,
        but heartbeats start, so that after a failure the survivors re-form a group among themselves
        (generation 0, 1, ...) instead of each training alone."""
        eg = cls(store, peer_id=f"r{rank}", backend=backend, **kw)
        eg.generation, eg.rank, eg.world_size = -1, int(rank), int(world_size)
        eg.members = [f"r{i}" for i in range(int(world_size))]
        return eg

    # -- membership -----------------------------------------------------------------------------------
    def _current_generation(self) -> int:
        return int(self.store.add("elastic/gen", 0))

    def join(self) -> int:
        """Join the current generation (or the next one if it already froze). Returns the rank."""
        while True:
            g = self._current_generation()
            ticket = int(self.store.add(f"elastic/g{g}/count", 1))
            self.store.set(f"elastic/g{g}/m{ticket}", self.peer_id)
            if ticket == 1:
                self._lead(g)
            self.store.wait([f"elastic/g{g}/frozen"], datetime.timedelta(seconds=self.matchmaking_time + 2 * self.timeout + 10))
            n = int(self.store.get(f"elastic/g{g}/frozen"))
            if ticket <= n:
                self.members = [self.store.get(f"elastic/g{g}/m{i}").decode() for i in range(1, n + 1)]
                self.generation, self.rank, self.world_size = g, ticket - 1, n
                break
            # arrived after the freeze: ask the members to open the next generation and wait for it
            self.store.set("elastic/join_pending", self.peer_id)
            self._wait_generation_after(g)
        self._init_group()
        logger.info(f"[elastic] {self.peer_id}: generation {self.generation}, rank {self.rank}/{self.world_size} "
                    f"members={self.members}")
        return self.rank

    def _lead(self, g: int):
        deadline = time.time() + self.matchmaking_time
        previous = [m for m in self.members if m != self.peer_id]  # members of the generation that failed
        while True:
            n = int(self.store.add(f"elastic/g{g}/count", 0))
            if time.time() >= deadline:
                if not previous:  # the first formation: wait for min_peers
                    done = n >= self.min_peers
                else:  # wait for every previous member that is still alive (fresh heartbeat), but not for a
                    # straggler past allreduce_timeout: it is dropped from this generation and rejoins later
                    arrived = {self.store.get(f"elastic/g{g}/m{i}").decode() for i in range(1, n + 1)}
                    done = all(m in arrived or not self._alive(m) for m in previous) or \
                        time.time() >= deadline + self.timeout
                if done:
                    break
            time.sleep(0.05)
        # freeze: the count at this instant is the member list; later tickets go to the next generation
        self.store.set(f"elastic/g{g}/frozen", str(int(self.store.add(f"elastic/g{g}/count", 0))))

    def _wait_generation_after(self, g: int):
        t0 = time.time()
        while self._current_generation() <= g:
            if time.time() - t0 > 10 * (self.matchmaking_time + self.timeout):
                raise TimeoutError(f"[elastic] no new generation after {g}")
            time.sleep(0.05)

    def _init_group(self):
        pstore = dist.PrefixStore(f"elastic/g{self.generation}/pg", self.store)
        dist.init_process_group(self.backend, store=pstore, rank=self.rank, world_size=self.world_size,
                                timeout=datetime.timedelta(seconds=self.timeout))

    # -- failure / growth -----------------------------------------------------------------------------
    def regroup(self):
        """Abort the current communicator and rendezvous in the next generation with whoever is alive."""
        old = self.generation
        if dist.is_initialized():
            # ABORT first (ncclCommAbort: releases kernels stuck on a dead peer without waiting for them),
            # then drop the registry entry so the next generation can initialise the default group again
            abort_group()
            try:
                if dist.is_initialized():  # an abort may already have dropped the group from the registry
                    dist.destroy_process_group()
            except Exception as e:  # noqa: BLE001 - a broken group may fail to tear down cleanly
                logger.warning(f"[elastic] destroy_process_group: {e!r}")
        # first survivor to get here opens generation old+1 (compare-and-set: bumped exactly once)
        self.store.compare_set("elastic/gen", str(old), str(old + 1))
        if self.store.check(["elastic/join_pending"]):
            self.store.delete_key("elastic/join_pending")
        self.regroups += 1
        self.join()

    def join_requested(self) -> bool:
        """Local view of the join flag (one store round trip, no collective)."""
        return bool(self.store.check(["elastic/join_pending"]))

    def poll_join(self) -> bool:
        """Collective: True (on every member) if a peer asked to join; the caller then regroups. The
        collaborative optimizer folds this flag into its round-opening all-gather instead where it has one."""
        local = 1.0 if self.join_requested() else 0.0
        flag = torch.tensor([local], device=self.device)
        self.guarded(lambda: dist.all_reduce(flag, op=dist.ReduceOp.MAX, async_op=True))
        return bool(flag.item() > 0)

    def guarded(self, launch) -> None:
        """Run one async collective under the watchdog timeout; raises on peer death / timeout."""
        work = launch()
        if work is not None:
            work.wait(timeout=datetime.timedelta(seconds=self.timeout))

    def shutdown(self):
        self._hb_stop.set()
        if dist.is_initialized():
            dist.destroy_process_group()
