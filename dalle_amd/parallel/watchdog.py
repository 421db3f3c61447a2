"""Deadlines for the collaborative rounds on the default (torchrun, non-elastic) path.

hivemind gives up on an all-reduce after ``allreduce_timeout`` and on the whole averaging step after
``averaging_timeout`` (``arguments.py:66-74``); a failed round falls back to the peer's own gradients
and training goes on. An RCCL communicator has no such notion: a collective whose peer died waits
forever (until the NCCL/RCCL watchdog tears the whole process down). So the round runs under a
host-side deadline:

* the round's collectives are enqueued as usual (RCCL: asynchronous to the host; the compute stream
  is made to wait on the communication stream), then ONE event is recorded on the compute stream and
  polled until it completes or the deadline passes (gloo on CPU: collectives are synchronous and raise
  on a closed peer connection or the process-group timeout);
* on expiry the communicator is ABORTED (``ncclCommAbort`` through ``_abort_process_group``; a
  ``destroy_process_group`` would itself block on the stuck kernels), the caller restores its local
  gradients and the peer continues without the group (``CollaborativeOptimizer`` detaches, or an
  ``ElasticGroup`` rendezvouses a new generation).

The poll costs one host wait per averaging round (once per ``target_batch_size`` samples).
"""
from __future__ import annotations

import time
from typing import Optional

import torch
import torch.distributed as dist

from ..utils.logging import get_logger

logger = get_logger(__name__)


class CollectiveTimeout(RuntimeError):
    pass


class Deadline:
    def __init__(self, seconds: Optional[float]):
        self.seconds = seconds
        self.t_end = None if seconds is None or seconds <= 0 else time.monotonic() + float(seconds)

    def remaining(self) -> float:
        return float("inf") if self.t_end is None else self.t_end - time.monotonic()

    def expired(self) -> bool:
        return self.t_end is not None and time.monotonic() > self.t_end


def wait_device(device: torch.device, deadline: Deadline, what: str = "collective") -> None:
    """Block the host until everything queued on the current stream so far has run (RCCL collectives
    included, through their stream dependency), or raise :class:`CollectiveTimeout`."""
    if torch.device(device).type != "cuda":
        return
    ev = torch.cuda.Event()
    ev.record()
    nap = 20e-6
    while not ev.query():
        if deadline.expired():
            raise CollectiveTimeout(f"{what} did not finish within {deadline.seconds:.1f} s")
        time.sleep(nap)
        nap = min(nap * 2, 2e-3)


def abort_group(group=None) -> None:
    """Abort the communicator of ``group`` (default: WORLD) without waiting for in-flight work."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    try:
        dist.distributed_c10d._abort_process_group(group if group is not None else dist.group.WORLD)
        return
    except Exception as e:  # noqa: BLE001 - older/other backends: fall back to the backend object
        logger.debug(f"_abort_process_group: {e!r}")
    try:
        pg = group if group is not None else dist.group.WORLD
        pg.abort()
    except Exception as e:  # noqa: BLE001
        logger.warning(f"could not abort the process group: {e!r}")
