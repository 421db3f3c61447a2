"""Fault injection and debug hooks (SURVEY §5.2-§5.3, §4 tier 5).

Configured by environment variables, checked at named injection points in the collaborative
optimizer and the trainer (all no-ops when unset):

* ``DALLE_AMD_FAULT_NAN_PARAMS=<epoch>``   -- overwrite one parameter with NaN after that epoch's update
                                              (exercises the callback's NaN rollback to ``state_path``)
* ``DALLE_AMD_FAULT_NAN_GRADS=<local step>`` -- poison the gradients at that local step
* ``DALLE_AMD_FAULT_DELAY_AVERAGING=<secs>`` -- sleep before every averaging round (slow peer)
* ``DALLE_AMD_FAULT_FAIL_AVERAGING=<epoch>``  -- raise inside the averaging round of that epoch
                                              (exercises the fall-back-to-local-gradients path)
* ``DALLE_AMD_FAULT_KILL_AT_EPOCH=<epoch>``  -- hard-exit the process (dead peer)
* ``DALLE_AMD_FAULT_KILL_IN_AVERAGING=<epoch>`` -- hard-exit inside that epoch's averaging round, after the
                                              round opened (the survivors are already in the collective)
* ``DALLE_AMD_DEBUG_SYNC=1``                 -- synchronise the device after every fused op (debug mode;
                                              pairs with ``AMD_SERIALIZE_KERNEL=3`` / ``HIP_LAUNCH_BLOCKING=1``)

Under torchrun every worker inherits the same environment; ``DALLE_AMD_FAULT_RANK=<r>`` limits the faults to
that ``RANK`` and ``DALLE_AMD_FAULT_ATTEMPT=<a>`` to that ``TORCHELASTIC_RESTART_COUNT`` (e.g. kill rank 1
in the first attempt only, then let ``--max-restarts`` bring the world back).
"""
from __future__ import annotations

import os
import time

import torch


def _targeted() -> bool:
    r, a = os.environ.get("DALLE_AMD_FAULT_RANK"), os.environ.get("DALLE_AMD_FAULT_ATTEMPT")
    if r not in (None, "") and os.environ.get("RANK", "0") != r:
        return False
    if a not in (None, "") and os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") != a:
        return False
    return True


def _int(name):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") and _targeted() else None


def debug_sync():
    if os.environ.get("DALLE_AMD_DEBUG_SYNC") == "1" and torch.cuda.is_available():
        torch.cuda.synchronize()


def before_averaging(epoch: int):
    d = os.environ.get("DALLE_AMD_FAULT_DELAY_AVERAGING")
    if d:
        time.sleep(float(d))
    if _int("DALLE_AMD_FAULT_KILL_IN_AVERAGING") == epoch:
        os._exit(17)
    if _int("DALLE_AMD_FAULT_FAIL_AVERAGING") == epoch:
        raise RuntimeError(f"injected averaging failure at epoch {epoch}")


@torch.no_grad()
def after_update(epoch: int, params):
    if _int("DALLE_AMD_FAULT_NAN_PARAMS") == epoch:
        p = next(iter(params))
        p.view(-1)[0] = float("nan")
    if _int("DALLE_AMD_FAULT_KILL_AT_EPOCH") == epoch:
        os._exit(17)


@torch.no_grad()
def on_local_step(step: int, params):
    if _int("DALLE_AMD_FAULT_NAN_GRADS") == step:
        for p in params:
            if p.grad is not None:
                p.grad.fill_(float("nan"))
                break
