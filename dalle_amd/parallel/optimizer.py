"""The collaborative optimizer: hivemind.Optimizer semantics on RCCL collectives.

Normative behaviour (``task.py:127-134``, ``arguments.py:59-78``):

1. Local accumulation: every ``.step()`` adds ``batch_size_per_step`` samples; gradients accumulate in
   ``.grad`` (``reuse_grad_buffers``: the trainer's ``zero_grad`` is bypassed) or in separate buffers.
2. Epoch trigger: when the peers together accumulated ``target_batch_size`` samples.
3. Gradient averaging: ``G = sum_p s_p * (g_p / t_p) / sum_p s_p`` (sample-weighted mean of per-peer
   mean gradients) -- plain RCCL all-reduce, compressed butterfly all-reduce (fp16 / uniform 8-bit,
   ``averaging.py``) or PowerSGD rank-r (``powersgd.py``). On failure a peer keeps its own ``g_p / t_p``.
4. Optimizer step (inner optimizer, e.g. fused 8-bit LAMB with global clipping), ``scheduler.step()``,
   ``local_epoch += 1``.
5. State averaging every ``average_state_every`` epochs (parameters, optionally compressed).
6. Reset accumulators.
7. Resync: a peer whose epoch lags the collaboration loads the state from a donor peer.

Peers are the ranks of a ``torch.distributed`` process group (backend "nccl" = RCCL over xGMI on a
MI355X node; "gloo" for CPU peers). Progress is asynchronous (``progress.py``, mode ``store``): every
peer adds its samples to a per-epoch counter in the job's key/value store and accumulates at its own
pace; whoever sees the total reach ``target_batch_size`` enters the round. The round opens with ONE
tiny all-gather of every peer's ``(samples, epoch)`` -- the exact weights, and a collective decision
on resynchronising lagging peers -- so the static RCCL communicator replaces hivemind's matchmaking.
Homogeneous nodes may use mode ``static`` (no communication outside the averaging itself).

Deadlines (``watchdog.py``): the averaging round runs under ``averaging_timeout``; on expiry or a dead
peer the communicator is aborted, the peer keeps its own gradients and parameters for that epoch and
continues without the group (or re-forms one through an ``ElasticGroup``).
"""
from __future__ import annotations

import time
from typing import Callable, Iterable, List, Optional, Union

import torch
import torch.distributed as dist

from .averaging import allreduce_weighted
from .compression import CompressionBase, NoCompression
from .delayed import AsyncStep, MasterParams
from .powersgd import PowerSGD
from .progress import ProgressTracker
from .watchdog import Deadline, abort_group, wait_device
from ..optim.flat import FlatArena
from ..utils import faults
from ..utils.logging import get_logger

logger = get_logger(__name__)


def _segments_of(tensors) -> List[tuple]:
    """``(offset, numel)`` of tensors packed back to back (``torch.cat`` of their flattened views)."""
    out, off = [], 0
    for t in tensors:
        out.append((off, t.numel()))
        off += t.numel()
    return out


def _group_world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


class GradientAverager:
    """Accumulates local gradients and averages them across peers (D15)."""

    def __init__(self, params: List[torch.nn.Parameter], arena: Optional[FlatArena] = None, group=None,
                 reuse_grad_buffers: bool = False, compression: Optional[CompressionBase] = None,
                 powersgd: Optional[PowerSGD] = None, client_mode: bool = False,
                 averaging_timeout: Optional[float] = None):
        self.params = params
        self.arena = arena
        self.group = group
        self.reuse_grad_buffers = reuse_grad_buffers
        self.compression = compression or NoCompression()
        self.powersgd = powersgd
        self.client_mode = client_mode
        self.averaging_timeout = averaging_timeout
        self.local_samples_accumulated = 0
        self.local_times_accumulated = 0
        self._acc: Optional[List[torch.Tensor]] = None
        self.last_averaging_ok = True
        self.last_round_exact = False  # the last round was an uncompressed all-reduce that succeeded
        self.detached = False          # the communicator was aborted: this peer continues alone
        self.comm_failed = False       # set when a collective failed (timeout / dead peer)
        self._backup_buf: Optional[torch.Tensor] = None  # one preallocated restore buffer (no clone per round)
        self._overlap = None           # GradSync: the round's all-reduce launched from inside backward
        self._armed = False
        self.overlapped_rounds = 0

    def _world(self):
        return (1, 0) if self.detached else _group_world(self.group)

    # -- accumulation -----------------------------------------------------------------------------
    @torch.no_grad()
    def accumulate_grads_(self, batch_size: int):
        self.local_samples_accumulated += int(batch_size)
        self.local_times_accumulated += 1
        if self.reuse_grad_buffers:
            return
        if self._acc is None:
            self._acc = [torch.zeros_like(p, dtype=torch.float32) for p in self.params]
        for a, p in zip(self._acc, self.params):
            if p.grad is not None:
                a.add_(p.grad)

    def _backup_of(self, flat: torch.Tensor) -> torch.Tensor:
        """Copy of ``flat`` in a buffer allocated once (a failed round restores from it)."""
        if self._backup_buf is None or self._backup_buf.shape != flat.shape or self._backup_buf.device != flat.device:
            self._backup_buf = torch.empty_like(flat)
        self._backup_buf.copy_(flat)
        return self._backup_buf

    # -- backward-overlapped rounds ------------------------------------------------------------------
    def overlap_eligible(self) -> bool:
        return (self.arena is not None and self.reuse_grad_buffers and self.powersgd is None
                and isinstance(self.compression, NoCompression) and not self.detached and self._world()[0] > 1)

    @torch.no_grad()
    def arm(self, next_closes_round: bool):
        """Called between micro-steps: if the NEXT backward completes this epoch's accumulation, hand the
        fused backward a GradSync hook so every gradient range that becomes final during that backward is
        all-reduced right away, overlapped with the remaining layers (parallel/dp.py) -- the round itself
        then only sends the tail (tied head, final LN) and rescales. Uncompressed rounds of homogeneous
        peers only (equal samples per peer: the sum over peers / (t * world) is the weighted mean)."""
        if not next_closes_round or not self.overlap_eligible():
            self.disarm()
            return
        if self._armed:
            return
        from .dp import GradSync

        if self._overlap is None or self._overlap.group is not self.group:
            self._overlap = GradSync(self.arena, world_size=self._world()[0], group=self.group, average=False)
        # the grads accumulated so far: a failed round falls back to them (the closing micro-batch is dropped)
        self._backup_of(self.arena.grad)
        self._overlap.attach()
        self._armed = True

    def disarm(self):
        if self._overlap is not None:
            self._overlap.detach()
        self._armed = False

    @torch.no_grad()
    def abandon_overlap(self):
        """A round that will not average (overflow skip, resync): complete the collectives the backward
        already launched -- every peer launched the same ones -- and drop the hook; the caller resets
        the accumulated gradients."""
        if self._armed:
            try:
                self._overlap.all_reduce()
            except Exception as e:  # noqa: BLE001
                logger.warning(f"abandoned overlapped round failed ({e!r})")
                self.comm_failed = True
                self._overlap._works, self._overlap._sent = [], []
        self.disarm()

    @torch.no_grad()
    def _step_overlapped(self, epoch: int, batch_size: int) -> bool:
        """Finish a round whose all-reduce was launched from inside the last backward."""
        sync, self._armed = self._overlap, False
        sync.detach()
        world, _ = self._world()
        t = max(1, self.local_times_accumulated)
        g = self.arena.grad
        deadline = Deadline(self.averaging_timeout)
        try:
            faults.before_averaging(epoch)
            sync.all_reduce()  # the tail + wait (the backward-launched buckets are already in flight)
            wait_device(g.device, deadline, "gradient averaging")
            g.mul_(1.0 / (t * world))
            self.overlapped_rounds += 1
            self.last_averaging_ok, self.last_round_exact = True, True
            return True
        except Exception as e:  # noqa: BLE001
            logger.warning(f"gradient averaging failed ({e!r}); falling back to local gradients "
                           f"(without the closing micro-batch, whose grads were already in the collective)")
            self.comm_failed = True  # the group's collectives were in flight: it must be re-formed / left
            sync._works, sync._sent = [], []
            g.copy_(self._backup_buf)
            self.local_times_accumulated = max(1, t - 1)
            self.local_samples_accumulated = max(0, self.local_samples_accumulated - int(batch_size))
            g.div_(self.local_times_accumulated)
            self.last_averaging_ok, self.last_round_exact = False, False
            return False

    def _grads(self) -> List[torch.Tensor]:
        if self.reuse_grad_buffers:
            for p in self.params:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
            return [p.grad for p in self.params]
        return self._acc if self._acc is not None else [torch.zeros_like(p) for p in self.params]

    # -- averaging --------------------------------------------------------------------------------
    @torch.no_grad()
    def step(self, total_samples: Optional[int] = None, epoch: int = 0, batch_size: int = 0) -> bool:
        """Replace the accumulated grads with the collaboration-wide weighted mean (in the params'
        ``.grad``). Returns False if averaging failed and this peer's own mean gradient was used."""
        if self._armed:
            return self._step_overlapped(epoch, batch_size)
        t = max(1, self.local_times_accumulated)
        s = float(self.local_samples_accumulated)
        world, _ = self._world()
        grads = self._grads()
        ok, exact = True, False
        if world == 1:
            try:
                faults.before_averaging(epoch)
            except Exception as e:  # noqa: BLE001
                logger.warning(f"gradient averaging failed ({e!r}); falling back to local gradients")
                ok = False
            for g in grads:
                g.div_(t)
        else:
            flat, views = self._flat(grads)  # x_p = this peer's MEAN gradient (g_p / t_p), one flat buffer
            try:
                faults.before_averaging(epoch)
                injected = False
            except Exception as e:  # noqa: BLE001 - an injected failure happens before any collective
                logger.warning(f"gradient averaging failed ({e!r}); falling back to local gradients")
                ok, injected = False, True
            if not injected:
                backup = self._backup_of(flat)
                deadline = Deadline(self.averaging_timeout)
                try:
                    if self.powersgd is not None:
                        total = float(total_samples) if total_samples else None
                        if total is None:
                            tt = torch.tensor([s], device=flat.device, dtype=torch.float32)
                            dist.all_reduce(tt, group=self.group)
                            total = float(tt.item())
                        saved_grads = None
                        if views is not None:  # PowerSGD reads and writes the params' .grad
                            self._unflat(flat, views)
                            # temporary .grad bindings: without reuse_grad_buffers `views` are the
                            # accumulators, and leaving them bound as .grad would alias p.grad with its
                            # own accumulator (the next accumulate_grads_ would add it into itself)
                            saved_grads = [p.grad for p in self.params]
                            for p, g in zip(self.params, views):
                                p.grad = g
                        try:
                            self.powersgd.allreduce_(scale=s * world / max(total, 1e-30))
                        finally:
                            if saved_grads is not None:
                                for p, g0 in zip(self.params, saved_grads):
                                    p.grad = g0
                        if views is not None:
                            flat, views = self._flat_nodiv(grads), grads
                    else:
                        shards = None if isinstance(self.compression, NoCompression) else self._shard_weights(world)
                        segs = self.arena.segments() if views is None else _segments_of(views)
                        allreduce_weighted(flat, weight=s, group=self.group, compression=self.compression,
                                           shard_weights=shards, total_weight=total_samples, segments=segs)
                        exact = isinstance(self.compression, NoCompression)
                    wait_device(flat.device, deadline, "gradient averaging")
                except Exception as e:  # noqa: BLE001 - a dead / slow peer must not kill training
                    logger.warning(f"gradient averaging failed ({e!r}); falling back to local gradients")
                    ok, exact = False, False
                    self.comm_failed = True
                    flat.copy_(backup)
            if views is not None:
                self._unflat(flat, views)
        if not self.reuse_grad_buffers:
            for p, g in zip(self.params, grads):
                if p.grad is None:
                    p.grad = g.clone()
                else:
                    p.grad.copy_(g)
        self.last_averaging_ok = ok
        self.last_round_exact = exact
        return ok

    def _shard_weights(self, world: int):
        """Butterfly shard sizes: client-mode peers host no shard (D17). Gathered once, then cached."""
        if world == 1:
            return None
        if getattr(self, "_shards", None) is None:
            flags = torch.tensor([0.0 if self.client_mode else 1.0], device=self._device())
            allf = [torch.zeros_like(flags) for _ in range(world)]
            dist.all_gather(allf, flags, group=self.group)
            self._shards = [float(f.item()) for f in allf]
        return self._shards

    def _device(self):
        return self.params[0].device

    def _flat(self, grads):
        """Per-peer mean gradient as one flat buffer (the arena's grad buffer when available)."""
        t = max(1, self.local_times_accumulated)
        if self.arena is not None and self.reuse_grad_buffers:
            self.arena.grad.div_(t)
            return self.arena.grad, None
        for g in grads:
            g.div_(t)
        return self._flat_nodiv(grads), grads

    @staticmethod
    def _flat_nodiv(grads):
        return torch.cat([g.reshape(-1).float() for g in grads])

    @staticmethod
    def _unflat(flat, views):
        off = 0
        for g in views:
            k = g.numel()
            g.copy_(flat[off:off + k].view_as(g))
            off += k

    @torch.no_grad()
    def reset_accumulated_grads_(self):
        self.local_samples_accumulated = 0
        self.local_times_accumulated = 0
        if self.arena is not None and self.reuse_grad_buffers:
            self.arena.zero_grad()
        else:
            for p in self.params:
                if p.grad is not None:
                    p.grad.zero_()
            if self._acc is not None:
                for a in self._acc:
                    a.zero_()


class TrainingStateAverager:
    """Holds the inner optimizer + scheduler, the local epoch, and averages parameters (D16).

    With ``master`` (a ``MasterParams``) the inner optimizer steps on master copies (hivemind's
    ``offload_optimizer``); with ``delay`` the step itself runs concurrently with the next local
    step (``delay_optimizer_step``, see ``delayed.py``) and is applied to the model -- followed by
    the state-averaging round of that epoch -- at the next ``finish_pending`` boundary.

    State averaging re-converges replicas that drifted (compressed or failed gradient rounds). After an
    EXACT round (uncompressed RCCL all-reduce: every peer received bit-identical averaged gradients and
    applied the same deterministic update to identical parameters) the replicas are already identical,
    so the round is skipped when ``skip_if_exact`` ("skip when all peers apply identical
    updates") -- on every peer alike, since the exactness flag is the same on all of them."""

    def __init__(self, optimizer: torch.optim.Optimizer, scheduler=None, params=None, arena: Optional[FlatArena] = None,
                 group=None, compression: Optional[CompressionBase] = None, average_state_every: int = 1,
                 master: Optional[MasterParams] = None, delay: bool = False, averaging_timeout: Optional[float] = None,
                 skip_if_exact: bool = True, check_every: int = 16):
        self.optimizer = optimizer
        self.scheduler = scheduler
        self.params = params
        self.arena = arena
        self.group = group
        self.compression = compression or NoCompression()
        self.average_state_every = average_state_every
        self.local_epoch = 0
        self.master = master
        self.runner = AsyncStep(master.masters[0].device) if (delay and master is not None and master.masters) else None
        self.averaging_timeout = averaging_timeout
        self.skip_if_exact = skip_if_exact
        self.check_every = int(check_every)  # verify the "replicas are identical" assumption this often
        self.drift_detected = 0
        self.detached = False
        self.comm_failed = False
        self.rounds_skipped = 0
        self._unapplied = False      # an update exists in the master copy but not in the model yet
        self._averaging_due = False  # the state-averaging round of the last delayed epoch has not run yet
        self._exact = False          # the gradient round of the pending epoch was exact
        self._backup_buf: Optional[torch.Tensor] = None  # restore buffer of a failed round, allocated once

    def _inner_step(self):
        self.optimizer.step()
        if self.scheduler is not None:
            self.scheduler.step()

    @torch.no_grad()
    def step(self, optimizer_step: bool = True, averaging_round: bool = True, exact: bool = False):
        self._exact = bool(exact)
        if optimizer_step:
            self.finish_pending(average=False)
            if self.master is not None:
                self.master.pull()
            if self.runner is not None:
                self.runner.launch(self._inner_step)
                self._unapplied = True
                self._averaging_due = averaging_round
                self.local_epoch += 1
                return
            self._inner_step()
            if self.master is not None:
                self.master.push()
            self.local_epoch += 1
        if averaging_round and self.average_state_every and self.local_epoch % self.average_state_every == 0:
            self.average_parameters()

    @property
    def pending(self) -> bool:
        return self._unapplied or self._averaging_due

    @torch.no_grad()
    def finish_pending(self, average: bool = True) -> bool:
        """Apply an in-flight delayed update to the model. ``average=True`` (the collective boundary,
        reached by every peer at its next ``.step()``) also runs that epoch's state-averaging round;
        local callers (``state_dict``, backups) pass False and leave the round to the boundary.
        Returns True if an update was applied."""
        applied = False
        if self._unapplied:
            self.runner.wait()
            self.master.push()
            self._unapplied = False
            applied = True
        if average and self._averaging_due:
            self._averaging_due = False
            if self.average_state_every and self.local_epoch % self.average_state_every == 0:
                self.average_parameters()
        return applied

    @torch.no_grad()
    def drop_pending(self):
        """Discard an in-flight update (the model state is being replaced from a backup / a peer).
        The epoch's averaging round stays due: it is a collective every peer must join."""
        if self.runner is not None:
            self.runner.wait()
        self._unapplied = False

    @torch.no_grad()
    def _replicas_differ(self) -> bool:
        if self.arena is not None:
            data = self.arena.data
        else:
            data = torch.cat([p.detach().reshape(-1).float() for p in self.params])
        h = data.view(torch.int32).sum(dtype=torch.int64)
        v = torch.stack([h, -h])  # int64: exact
        try:
            dist.all_reduce(v, op=dist.ReduceOp.MAX, group=self.group)  # (max, -min) of the checksum
        except Exception as e:  # noqa: BLE001
            logger.warning(f"replica check failed ({e!r})")
            self.comm_failed = True
            return False
        return bool(v[0].item() != -v[1].item())

    @torch.no_grad()
    def average_parameters(self):
        world, _ = (1, 0) if self.detached else _group_world(self.group)
        if world == 1:
            return
        if self.skip_if_exact and self._exact:
            # the skip assumes every peer ran the same deterministic update on identical parameters; every
            # `check_every` epochs that is VERIFIED with one 2-element all-reduce of an exact parameter
            # checksum (integer sum of the fp32 bit patterns), and a real round runs if replicas drifted
            if not (self.check_every > 0 and self.local_epoch % self.check_every == 0 and self._replicas_differ()):
                self.rounds_skipped += 1
                return
            self.drift_detected += 1
            logger.warning(f"replica parameters differ after an exact round (epoch {self.local_epoch}); averaging them")
        buf = self.arena.data if self.arena is not None else torch.cat([p.detach().reshape(-1).float() for p in self.params])
        segs = self.arena.segments() if self.arena is not None else _segments_of(self.params)
        if self._backup_buf is None or self._backup_buf.shape != buf.shape or self._backup_buf.device != buf.device:
            self._backup_buf = torch.empty_like(buf)
        backup = self._backup_buf
        backup.copy_(buf)
        deadline = Deadline(self.averaging_timeout)
        try:
            allreduce_weighted(buf, 1.0, self.group, self.compression, total_weight=float(world), segments=segs)
            wait_device(buf.device, deadline, "state averaging")
        except Exception as e:  # noqa: BLE001
            logger.warning(f"state averaging failed ({e!r}); keeping local parameters")
            self.comm_failed = True
            buf.copy_(backup)
        if self.arena is None:
            off = 0
            for p in self.params:
                k = p.numel()
                p.data.copy_(buf[off:off + k].view_as(p))
                off += k


class CollaborativeOptimizer(torch.optim.Optimizer):
    """Drop-in for ``hivemind.Optimizer`` as constructed at ``task.py:127-134``."""

    def __init__(self, *, dht=None, run_id: str, params: Union[Iterable, List[dict]],
                 optimizer: Union[Callable, torch.optim.Optimizer], scheduler: Optional[Callable] = None,
                 target_batch_size: int, batch_size_per_step: Optional[int] = None, matchmaking_time: float = 15.0,
                 allreduce_timeout: float = 60.0, averaging_timeout: float = 180.0, offload_optimizer: bool = False,
                 delay_grad_averaging: bool = False, delay_optimizer_step: bool = False, reuse_grad_buffers: bool = False,
                 grad_compression: Optional[CompressionBase] = None,
                 state_averaging_compression: Optional[CompressionBase] = None, average_state_every: int = 1,
                 client_mode: bool = False, auxiliary: bool = False, verbose: bool = False, process_group=None,
                 arena: Optional[FlatArena] = None, powersgd_rank: Optional[int] = None, tracker_mode: str = "auto",
                 device=None, elastic=None, skip_exact_state_averaging: bool = True, offload_device=None,
                 recovery: str = "auto", state_check_every: int = 16, overlap_grad_averaging: bool = True, **kwargs):
        self.dht, self.run_id = dht, run_id
        self.target_batch_size = target_batch_size
        self.batch_size_per_step = batch_size_per_step
        self.matchmaking_time, self.allreduce_timeout, self.averaging_timeout = matchmaking_time, allreduce_timeout, averaging_timeout
        self.offload_optimizer = offload_optimizer
        self.delay_grad_averaging, self.delay_optimizer_step = delay_grad_averaging, delay_optimizer_step
        self.client_mode, self.auxiliary, self.verbose = client_mode, auxiliary, verbose
        self.group = process_group
        self.arena = arena
        self.elastic = elastic  # ElasticGroup: survive peer death / admit joiners

        param_groups = list(params)
        if param_groups and isinstance(param_groups[0], dict):
            flat_params = [p for g in param_groups for p in g["params"]]
        else:
            flat_params = param_groups
            param_groups = [{"params": flat_params}]
        self._params = flat_params
        factory = callable(optimizer) and not isinstance(optimizer, torch.optim.Optimizer)
        if delay_optimizer_step and not factory:
            logger.warning("delay_optimizer_step needs an optimizer factory (it builds the optimizer over master "
                           "copies); stepping synchronously")
        # delayed update: the inner optimizer owns master copies (hivemind's offloaded parameters, kept in HBM)
        # offload_device="cpu": the master copy + optimizer state live in pinned host memory and the step
        # runs on the CPU (the reference's CPULAMB8Bit regime); default: an HBM master copy
        want_master = factory and flat_params and (delay_optimizer_step or offload_device is not None)
        self._master = MasterParams(flat_params, arena, device=offload_device) if want_master else None
        inner = optimizer(self._master.substitute(param_groups) if self._master else param_groups) if factory else optimizer
        if offload_device is not None and self._master is None and flat_params:
            # an already-built optimizer (no factory to rebuild it over MasterParams): step it on pinned
            # host copies through the generic wrapper
            from ..optim.wrapper import HostOffloadOptimizer
            inner = HostOffloadOptimizer(inner)
        if arena is not None and getattr(inner, "arena", "missing") is None:
            inner.arena = self._master.arena if self._master is not None else arena
        sched = scheduler(inner) if callable(scheduler) else scheduler
        device = device or (flat_params[0].device if flat_params else torch.device("cpu"))
        self.device = device
        peer_id = dht.peer_id if dht is not None else f"rank{_group_world(process_group)[1]}"
        # failure recovery on the default (static torchrun) world: with a store that outlives the trainers
        # (the torchrun agent's, or DALLE_AMD_COORDINATOR) the world is adopted as elastic generation -1,
        # so after a dead / timed-out peer the survivors re-form a group and keep averaging; without one
        # (or recovery="detach") a failed peer's survivors detach and train alone
        self.adopted = False
        tracker_store = None
        world0, rank0 = _group_world(process_group)
        if elastic is None and recovery == "auto" and world0 > 1 and (process_group is None or process_group == dist.group.WORLD):
            from .elastic import ElasticGroup, recovery_store
            rstore = recovery_store(run_id, timeout=max(30.0, float(averaging_timeout or 0)))
            if rstore is not None:
                elastic = ElasticGroup.adopt(rstore, rank0, world0, backend=dist.get_backend(),
                                             matchmaking_time=min(float(matchmaking_time), 15.0),
                                             allreduce_timeout=float(allreduce_timeout), device=device)
                self.elastic = elastic
                self.adopted = True
                tracker_store = dist.PrefixStore("progress", rstore)
        if elastic is not None and not self.adopted:
            # a peer that JOINS through the coordinator takes the tracker of the group it joins (an
            # adopted torchrun world publishes its mode; pure elastic generations default to lockstep)
            key = "elastic/tracker_mode"
            if tracker_mode == "auto":
                tracker_mode = elastic.store.get(key).decode() if elastic.store.check([key]) else "collective"
            if tracker_mode == "store":
                tracker_store = dist.PrefixStore("progress", elastic.store)
        if tracker_mode == "auto":
            # asynchronous store records on a static (or adopted) group
            tracker_mode = "store"
        if self.adopted:
            elastic.store.set("elastic/tracker_mode", tracker_mode)
        self.tracker = ProgressTracker(dht=dht, prefix=run_id, target_batch_size=target_batch_size, group=process_group,
                                       device=device, client_mode=client_mode, peer_id=peer_id, mode=tracker_mode,
                                       store=tracker_store)
        psgd = PowerSGD(flat_params, rank=powersgd_rank, group=process_group) if powersgd_rank else None
        self.grad_averager = GradientAverager(flat_params, arena=arena, group=process_group,
                                              reuse_grad_buffers=reuse_grad_buffers, compression=grad_compression,
                                              powersgd=psgd, client_mode=client_mode,
                                              averaging_timeout=averaging_timeout)
        self.state_averager = TrainingStateAverager(inner, sched, flat_params, arena=arena, group=process_group,
                                                    compression=state_averaging_compression,
                                                    average_state_every=average_state_every,
                                                    master=self._master, delay=delay_optimizer_step and self._master is not None,
                                                    averaging_timeout=averaging_timeout,
                                                    # the CPU-offloaded LAMB reduces with threads: not
                                                    # bitwise reproducible across peers, so never skip then
                                                    skip_if_exact=skip_exact_state_averaging and offload_device is None,
                                                    check_every=state_check_every)
        self.detached = False
        self.overlap_grad_averaging = overlap_grad_averaging
        # backward() calls per .step() (a trainer's gradient_accumulation_steps): the backward-overlapped
        # all-reduce needs exactly one, since the hook fires in every hooked backward
        self.backwards_per_step = 1
        self._join_seen: Optional[bool] = None
        self._last_bs = int(batch_size_per_step or 0)
        if self._last_bs:
            self._arm_next(self._last_bs)  # the very first micro-step may already close epoch 0
        self.last_round_samples = 0  # this peer's samples in the last averaging round
        self.last_epoch_time = None
        if offload_optimizer and device.type == "cuda" and verbose:
            where = "pinned host memory, CPU step" if (self._master is not None and self._master.offloaded) \
                else "an HBM master copy (fused HIP LAMB; 288 GB HBM)"
            logger.info(f"offload_optimizer=True: optimizer state in {where}")
        # torch.optim.Optimizer protocol (param_groups / state) for trainers and schedulers
        self.defaults = inner.defaults
        self._optimizer_step_pre_hooks = {}
        self._optimizer_step_post_hooks = {}

    # -- torch.optim.Optimizer protocol ------------------------------------------------------------
    @property
    def param_groups(self):
        return self.state_averager.optimizer.param_groups

    @property
    def state(self):
        return self.state_averager.optimizer.state

    @property
    def opt(self):
        return self.state_averager.optimizer

    @property
    def scheduler(self):
        return self.state_averager.scheduler

    @property
    def local_epoch(self) -> int:
        return self.state_averager.local_epoch

    @local_epoch.setter
    def local_epoch(self, v: int):
        self.state_averager.local_epoch = int(v)

    def zero_grad(self, set_to_none: bool = False):
        if self.grad_averager.reuse_grad_buffers:
            raise ValueError("zero_grad must not be called with reuse_grad_buffers=True: the optimizer zeroes "
                             "the accumulated gradients itself after each global step")
        for p in self._params:
            if p.grad is not None:
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.zero_()

    # -- main entry -----------------------------------------------------------------------------------
    def step(self, closure=None, batch_size: Optional[int] = None, grad_scaler=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if self.auxiliary:
            return loss
        self.finish_pending()
        self._local_steps = getattr(self, "_local_steps", 0) + 1
        faults.on_local_step(self._local_steps, self._params)
        bs = batch_size if batch_size is not None else self.batch_size_per_step
        if bs is None:
            raise ValueError("batch_size_per_step (ctor) or batch_size (step) is required")
        self.grad_averager.accumulate_grads_(bs)
        self._last_bs = int(bs)
        try:
            return self._step_collective(grad_scaler, loss)
        finally:
            self._arm_next(bs)

    def set_backwards_per_step(self, n: int):
        """Declare the number of backward() calls per .step() (gradient accumulation); anything but one
        disables the backward-overlapped all-reduce, which the hook would otherwise launch per backward."""
        self.backwards_per_step = max(1, int(n))
        if self.backwards_per_step != 1:
            self.grad_averager.disarm()
        elif self._last_bs:
            self._arm_next(self._last_bs)

    def _arm_next(self, bs: int):
        """Static homogeneous tracker: the next micro-step closes the epoch exactly when (accumulated +
        bs) * world >= target -- then its backward launches the round's all-reduce (GradientAverager.arm)."""
        ga = self.grad_averager
        if self.tracker.mode != "static" or self.detached or not self.overlap_grad_averaging \
                or int(getattr(self, "backwards_per_step", 1)) != 1:
            ga.disarm()
            return
        world = _group_world(self.group)[0]
        ga.arm((ga.local_samples_accumulated + int(bs)) * world >= self.target_batch_size)

    def _step_collective(self, grad_scaler, loss):
        if self.elastic is None:
            try:
                self._collective_part(grad_scaler)
            except Exception as e:  # noqa: BLE001 - the round's own collectives (boundary sync, resync)
                logger.warning(f"{self.run_id}: collective failure ({e!r})")
                self.grad_averager.comm_failed = True
            if self._comm_failed():
                self.detach()
            return loss
        try:
            self._collective_part(grad_scaler)
            if self._comm_failed() or not self.grad_averager.last_averaging_ok:
                raise RuntimeError("gradient averaging failed")
        except Exception as e:  # noqa: BLE001 - a member died / timed out: re-form the group and go on
            logger.warning(f"{self.run_id}: collective failure ({e!r}); regrouping")
            self._regroup()
        return loss

    def _comm_failed(self) -> bool:
        return self.grad_averager.comm_failed or self.state_averager.comm_failed

    def detach(self):
        """The communicator is broken (a peer died or missed the deadline): abort it -- never block in a
        teardown -- and go on training alone; every later epoch is a local one (a failed
        round falls back to local gradients and still advances the epoch)."""
        if self.detached:
            return
        logger.warning(f"{self.run_id}: aborting the communicator; this peer continues without the collaboration")
        abort_group(self.group)
        self.detached = True
        self.grad_averager.detached = self.state_averager.detached = True
        self.grad_averager.comm_failed = self.state_averager.comm_failed = False
        self.tracker.mode = "local"

    def _collective_part(self, grad_scaler):
        self.tracker.report_local_progress(self.local_epoch, self.grad_averager.local_samples_accumulated)
        tr = self.tracker
        if tr.mode == "collective":
            # load_state_from_peers is a collective: decide on (min, max) epoch, which the lockstep
            # tracker's reduction gives every rank identically -- up-to-date ranks join as donors
            lagging = tr.min_epoch_seen is not None and tr.min_epoch_seen < tr.max_epoch_seen - 1
        else:
            lagging = tr.mode == "dht" and tr.max_epoch_seen > self.local_epoch + 1
        if lagging:
            logger.info(f"epochs {tr.min_epoch_seen if tr.mode == 'collective' else self.local_epoch}..{tr.max_epoch_seen} "
                        f"diverged (local {self.local_epoch}); loading state from the newest peer")
            self.grad_averager.abandon_overlap()
            self.load_state_from_peers()
            self.grad_averager.reset_accumulated_grads_()
            return
        if self.tracker.ready_to_update_epoch:
            self._update_global_epoch(grad_scaler)

    def _regroup(self):
        """New communicator over the live members, then one donor brings everyone (joiners, or
        survivors whose last step fell back to local gradients) to the same state."""
        self.elastic.regroup()
        if self.group is not None:  # the old group object died with its communicator: rebind to the new WORLD
            self.group = dist.group.WORLD
            self.grad_averager.group = self.state_averager.group = self.tracker.group = self.group
            if self.grad_averager.powersgd is not None:
                self.grad_averager.powersgd.group = self.group
        self.grad_averager._shards = None
        self.grad_averager.last_averaging_ok = True
        self.grad_averager.comm_failed = self.state_averager.comm_failed = False
        self.load_state_from_peers()

    def _round_sync(self):
        """Opening of an averaging round on the asynchronous tracker: ONE all-gather of every peer's
        ``(samples accumulated, local epoch)``. Returns ``(total samples, min epoch, max epoch, peers)`` --
        identical on every rank, so the weighting and the resync decision are collective."""
        world, _ = (1, 0) if self.detached else _group_world(self.group)
        s = float(self.grad_averager.local_samples_accumulated)
        self._join_seen = None
        if world == 1 or self.tracker.mode not in ("store", "dht"):
            gp = self.tracker.global_progress
            total = gp.samples_accumulated if world > 1 else s
            return total, self.local_epoch, self.local_epoch, max(1, gp.num_peers if world > 1 else 1)
        dt = torch.float64 if self.device.type == "cpu" else torch.float32
        # the third field is this peer's view of the elastic join flag: the round's one all-gather
        # replaces a separate per-round join poll (an all-reduce + host sync)
        join = 1.0 if (self.elastic is not None and self.elastic.join_requested()) else 0.0
        mine = torch.tensor([s, float(self.local_epoch), join], dtype=dt, device=self.device)
        out = torch.empty(world * 3, dtype=dt, device=self.device)
        deadline = Deadline(self.averaging_timeout)
        if self.device.type == "cuda":
            dist.all_gather_into_tensor(out, mine, group=self.group)
            wait_device(self.device, deadline, "round opening")
        else:
            work = dist.all_gather(list(out.chunk(world)), mine, group=self.group, async_op=True)
            work.wait(timeout=__import__("datetime").timedelta(seconds=max(1.0, deadline.remaining())))
        v = out.view(world, 3).tolist()
        total = sum(r[0] for r in v)
        epochs = [int(round(r[1])) for r in v]
        self._join_seen = any(r[2] > 0 for r in v)
        return total, min(epochs), max(epochs), world

    def _update_global_epoch(self, grad_scaler=None):
        t0 = time.perf_counter()
        total, min_epoch, max_epoch, peers = self._round_sync()
        if min_epoch < max_epoch - 1:
            # some peer fell behind (e.g. restored an old local backup): everyone joins the resync
            logger.info(f"{self.run_id}: epochs {min_epoch}..{max_epoch} diverged; resynchronising from the newest peer")
            self.grad_averager.abandon_overlap()
            self.load_state_from_peers()
            self.grad_averager.reset_accumulated_grads_()
            self.tracker.update_epoch(self.local_epoch)
            return
        averaged = None
        if grad_scaler is not None and grad_scaler.is_enabled():
            # deferred AMP unscale + collaboration-wide overflow check (D28): skip the whole update
            # (and the averaging round) if any peer's accumulated grads overflowed
            if self.grad_averager._armed:
                # the last backward already launched this round's all-reduce on the (scaled) arena grads:
                # RCCL is still reading and writing them, so finish the round first and unscale the
                # averaged grads (unscaling is linear; an overflow on any peer is non-finite in the sum)
                averaged = self.grad_averager.step(total_samples=total, epoch=self.local_epoch, batch_size=self._last_bs)
            flat = self.arena.grad if (self.arena is not None and self.grad_averager.reuse_grad_buffers) else None
            # after a failed overlapped round (dead / slow peer, deadline hit) the group's communicator is
            # broken: check the local fallback grads without a collective instead of queueing one behind it
            local_only = averaged is False or self._comm_failed()
            if not grad_scaler.unscale_and_check(self.grad_averager._grads(), flat_grad=flat, group=self.group,
                                                 local_only=local_only):
                logger.warning(f"{self.run_id}: non-finite scaled gradients at epoch {self.local_epoch}; skipping update")
                self.grad_averager.abandon_overlap()
                self.grad_averager.reset_accumulated_grads_()
                self.local_epoch = max_epoch + 1
                self.tracker.update_epoch(self.local_epoch)
                return
        ok = averaged if averaged is not None else \
            self.grad_averager.step(total_samples=total, epoch=self.local_epoch, batch_size=self._last_bs)
        exact = ok and self.grad_averager.last_round_exact and min_epoch == max_epoch
        self.state_averager.step(optimizer_step=True, averaging_round=True, exact=exact)
        if self.local_epoch < max_epoch + 1:  # a peer one epoch behind catches up on the count
            self.local_epoch = max_epoch + 1
        if not self.state_averager.pending:
            faults.after_update(self.local_epoch, self._params)
        self.last_round_samples = int(self.grad_averager.local_samples_accumulated)
        self.grad_averager.reset_accumulated_grads_()
        self.tracker.update_epoch(self.local_epoch)
        self.last_epoch_time = time.perf_counter() - t0
        if self.verbose:
            logger.info(f"{self.run_id}: epoch {self.local_epoch} (averaged {int(total)} samples across "
                        f"{peers} peers in {self.last_epoch_time * 1e3:.1f} ms)")
        # joiners are admitted at a round boundary that EVERY member passes through (training peers from
        # step(), finished peers from leave()), so the poll's all-reduce always matches; a failed round
        # regroups anyway -- never poll over a broken communicator
        if self.elastic is not None and not self._comm_failed() and self.grad_averager.last_averaging_ok \
                and (self._join_seen if self._join_seen is not None else self.elastic.poll_join()):
            logger.info(f"{self.run_id}: a peer asked to join; regrouping at epoch {self.local_epoch}")
            self._regroup()

    # -- delayed parameter update ---------------------------------------------------------------------
    def finish_pending(self) -> bool:
        """Step boundary of ``delay_optimizer_step``: the update launched at the previous global step
        lands in the model, then that epoch's state-averaging round runs. Every peer reaches this at
        its next ``.step()``; call it directly before reading the model after the last step."""
        applied = self.state_averager.finish_pending(average=True)
        if applied:
            faults.after_update(self.local_epoch, self._params)
        return applied

    def apply_pending(self) -> bool:
        """Local part of the boundary only (no collective): the model gets the latest update; the
        averaging round stays due for the next ``.step()``. Used before checkpoints and at exit."""
        applied = self.state_averager.finish_pending(average=False)
        if applied:
            faults.after_update(self.local_epoch, self._params)
        return applied

    # -- state --------------------------------------------------------------------------------------
    def state_dict(self) -> dict:
        self.apply_pending()  # model and optimizer state of the same epoch
        sd = self.opt.state_dict()
        sd["state"]["local_epoch"] = self.local_epoch
        return sd

    def load_state_dict(self, state_dict: dict):
        self.state_averager.drop_pending()
        sd = dict(state_dict)
        sd["state"] = dict(sd["state"])
        if "local_epoch" in sd["state"]:
            self.local_epoch = int(sd["state"].pop("local_epoch"))
        self.opt.load_state_dict(sd)

    @torch.no_grad()
    def load_state_from_peers(self, **kwargs) -> bool:
        """Collective: every rank participates; the donor is the rank with the highest epoch
        (lowest rank on ties). Broadcasts parameters, optimizer state, scheduler state, epoch (C3)."""
        world, rank = _group_world(self.group)
        if world == 1:
            return False
        self.apply_pending()  # the donor ships its newest parameters
        dev = self.device
        score = torch.tensor([float(self.local_epoch * world + (world - 1 - rank))], device=dev, dtype=torch.float64 if dev.type == "cpu" else torch.float32)
        dist.all_reduce(score, op=dist.ReduceOp.MAX, group=self.group)
        best = int(round(score.item()))
        donor = world - 1 - (best % world)
        donor_global = dist.get_global_rank(self.group, donor) if self.group is not None else donor
        if self.arena is not None:
            dist.broadcast(self.arena.data, src=donor_global, group=self.group)
        else:
            for p in self._params:
                dist.broadcast(p.data, src=donor_global, group=self.group)
        # optimizer + scheduler state: only the skeleton (scalars, hyper-parameters, tensor shapes / dtypes)
        # goes through pickle; the state tensors (8-bit moments, absmax, fp32 moments) are packed into one
        # flat buffer per dtype and broadcast as tensors on the group (RCCL over xGMI on the GPU)
        sd = self.state_dict() if rank == donor else None
        tensors: List[torch.Tensor] = []
        meta = [(_strip_tensors(sd, tensors), self.scheduler.state_dict() if self.scheduler is not None else None)
                if rank == donor else None]
        dist.broadcast_object_list(meta, src=donor_global, group=self.group, device=dev if dev.type == "cuda" else None)
        skeleton, sched = meta[0]
        specs = _tensor_specs(skeleton)
        received = _broadcast_state_tensors(tensors if rank == donor else None, specs, donor_global, self.group, dev)
        if rank != donor:
            tensors = list(received.items())
            by_id = dict(tensors)
            self.load_state_dict(_fill_tensors(skeleton, by_id))
            if self.scheduler is not None and sched is not None:
                self.scheduler.load_state_dict(sched)
        self.tracker.update_epoch(self.local_epoch)
        return rank != donor

    def leave(self, poll: float = 0.02):
        """A peer that finished training stays in the group until EVERY peer finished (asynchronous
        peers finish at different times; a static communicator cannot lose a member mid-round): it
        joins the remaining averaging rounds with zero samples -- receiving the averaged gradients and
        applying the same update -- and exits once all peers announced the end. The end decision is
        consistent: after the last peer announced, no peer adds samples, so the epoch counter is frozen."""
        world, _ = (1, 0) if self.detached else _group_world(self.group)
        if world == 1 or self.tracker.mode != "store":
            return
        store, done_key = self.tracker.store, f"{self.tracker._ns}/done"
        # the samples accumulated so far are already in the shared counter: they stay this peer's
        # contribution to the next round (dropping them would make the round's weights disagree with it)
        store.add(done_key, 1)
        while not self.detached:
            self.finish_pending()
            if self._comm_failed():
                self.detach()
                break
            self.tracker.report_local_progress(self.local_epoch, 0)
            if self.tracker.ready_to_update_epoch:
                try:
                    self._update_global_epoch()
                except Exception as e:  # noqa: BLE001
                    logger.warning(f"{self.run_id}: collective failure while leaving ({e!r})")
                    self.detach()
                continue
            if int(store.add(done_key, 0)) >= _group_world(self.group)[0]:  # (a regroup may have changed it)
                break
            time.sleep(poll)
        self.finish_pending()

    def shutdown(self):
        self.apply_pending()
        self.tracker.shutdown()


STATE_CHUNK_BYTES = 128 * 2 ** 20   # staging window of a state transfer (one per rank, reused)


def _broadcast_state_tensors(src, specs, donor_global, group, dev, chunk_bytes: int = None):
    """Broadcast the state tensors of a transfer from the donor (``src`` = its tensors, in ``specs`` order;
    None on receivers) in fixed windows: per dtype, the tensors form one virtual flat stream cut into windows of
    ``chunk_bytes``; the donor packs each window into a staging buffer, broadcasts it, and every receiver scatters
    it into the destination tensors it preallocated. The peak extra memory is one window per rank -- not a
    second copy of the whole optimizer state (8-bit moments + absmax + fp32 tensors: GBs at the 1.3B scale).
    Returns ``{index: tensor}`` on receivers, {} on the donor."""
    chunk_bytes = chunk_bytes or STATE_CHUNK_BYTES
    out = {}
    for dtype in sorted({sp[1] for sp in specs}, key=str):
        idx = [i for i, sp in enumerate(specs) if sp[1] == dtype]
        if not idx:
            continue
        total = sum(specs[i][2] for i in idx)
        win = max(1, chunk_bytes // torch.empty((), dtype=dtype).element_size())
        stage = torch.empty(min(win, total), dtype=dtype, device=dev)
        if src is None:
            for i in idx:
                out[i] = torch.empty(specs[i][0], dtype=dtype, device=dev)
        flats = [(src[i] if src is not None else out[i]).reshape(-1) for i in idx]
        starts, acc = [], 0
        for i in idx:
            starts.append(acc)
            acc += specs[i][2]
        for w0 in range(0, total, win):
            w1 = min(total, w0 + win)
            pieces = []   # (flat tensor, its [a, b) range, the window offset)
            for f, st in zip(flats, starts):
                a, b = max(w0, st), min(w1, st + f.numel())
                if a < b:
                    pieces.append((f, a - st, b - st, a - w0))
            buf = stage[:w1 - w0]
            if src is not None:
                for f, a, b, o in pieces:
                    buf[o:o + b - a].copy_(f[a:b].detach())
            dist.broadcast(buf, src=donor_global, group=group)
            if src is None:
                for f, a, b, o in pieces:
                    f[a:b].copy_(buf[o:o + b - a])
    return out


class _TensorSlot:
    """Placeholder for a state tensor in the pickled skeleton of a state transfer."""

    def __init__(self, idx: int, shape, dtype):
        self.idx, self.shape, self.dtype = idx, tuple(shape), dtype


def _strip_tensors(obj, out: list):
    if torch.is_tensor(obj):
        out.append(obj)
        return _TensorSlot(len(out) - 1, obj.shape, obj.dtype)
    if isinstance(obj, dict):
        return {k: _strip_tensors(v, out) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_strip_tensors(v, out) for v in obj)
    return obj


def _tensor_specs(obj, acc=None):
    """(shape, dtype, numel) of every slot, indexed by slot id."""
    acc = {} if acc is None else acc
    if isinstance(obj, _TensorSlot):
        n = 1
        for d in obj.shape:
            n *= d
        acc[obj.idx] = (obj.shape, obj.dtype, n)
    elif isinstance(obj, dict):
        for v in obj.values():
            _tensor_specs(v, acc)
    elif isinstance(obj, (list, tuple)):
        for v in obj:
            _tensor_specs(v, acc)
    return [acc[i] for i in range(len(acc))]


def _fill_tensors(obj, by_id: dict):
    if isinstance(obj, _TensorSlot):
        return by_id[obj.idx]
    if isinstance(obj, dict):
        return {k: _fill_tensors(v, by_id) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_fill_tensors(v, by_id) for v in obj)
    return obj


def _to_cpu(obj):
    if torch.is_tensor(obj):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _to_cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_cpu(v) for v in obj)
    return obj


# hivemind name
Optimizer = CollaborativeOptimizer
