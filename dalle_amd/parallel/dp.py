"""Data-parallel gradient synchronisation over RCCL (xGMI) / gloo.

The gradient arena is one contiguous buffer (``FlatArena``), so a bucket is just a slice: no pack /
unpack copies. Buckets are sized for the xGMI mesh: each of the 8 GPUs has 7
point-to-point links; RCCL splits an all-reduce into per-peer slices, and a 64 MB bucket keeps each
per-link slice at >= 4 MB, past the latency-bound regime, while still pipelining several
collectives.

Overlap with backward (``attach()``): the fused stacks' backward (``hip_ops._SequentialFused`` /
``_ReversibleFused``) reports the parameters whose arena grads have just become final -- a layer's
own weights right after its backward in an unshared model (the 1.3B preset), a shared block's after
the LAST layer that reuses it (the first in forward order) -- and ``notify`` launches their
all-reduce right there, asynchronously: RCCL's stream waits for the kernels that produced those grads
and then runs beside the remaining backward layers. ``all_reduce()`` after ``backward()`` only sends
what is left (tied embedding / head, final LayerNorm) and waits. In the bench24 / reference presets
(5 blocks reused by every layer) two thirds of the bytes become final during the last five layers'
backward; in an unshared model almost everything overlaps. Requires one ``all_reduce()`` per
``backward()`` (no local accumulation across micro-batches while attached).

``algo``: ``"rccl"`` runs one ``all_reduce`` per bucket (RCCL picks ring / tree over the xGMI mesh);
``"rs_ag"`` runs the direct mesh form of SURVEY §5.8 explicitly -- per bucket a ``reduce_scatter_tensor``
(each rank reduces 1/N of the bucket, with the 1/N average fused into the reduction as RCCL's ``AVG`` op
where it applies) followed by an ``all_gather_into_tensor`` of the reduced shards. Every rank then holds
the SAME bits for every element (each shard is reduced once, by one rank).

``grad_dtype='bf16'`` halves the bytes on the wire (RCCL then reduces in bf16, so the averaged gradient
carries bf16 rounding -- use for large worlds only). It overlaps with backward too: ``notify`` casts each
final range into the preallocated bf16 wire buffer and launches its collective there; ``all_reduce()``
copies the reduced ranges back.

Neither the bucket size nor the algorithm is a guess for a given mesh: ``tune_grad_sync`` times the full
arena all-reduce for every (algorithm, bucket size) candidate on the real communicator (max over ranks,
so every rank picks the same one) and bench.py uses the fastest (``--allreduce-algo auto``).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..optim.flat import FlatArena

DEFAULT_BUCKET_BYTES = 64 * 1024 * 1024


class GradSync:
    def __init__(self, arena: FlatArena, world_size: int = 1, group=None, grad_dtype: str = "fp32",
                 bucket_bytes: int = DEFAULT_BUCKET_BYTES, average: bool = True, algo: str = "rccl"):
        if algo not in ("rccl", "rs_ag"):
            raise ValueError(f"unknown all-reduce algorithm {algo!r} (rccl | rs_ag)")
        self.algo = algo
        self.arena = arena
        self.world_size = world_size
        self.group = group
        self.grad_dtype = grad_dtype
        self.average = average
        self.bucket_elems = max(1, int(bucket_bytes) // 4)
        elems = self.bucket_elems
        self.buckets = [(s, min(s + elems, arena.numel)) for s in range(0, arena.numel, elems)]
        self._lowp = None
        self._range = {id(p): (o, (p.numel() + arena.align - 1) // arena.align * arena.align)
                       for p, o in zip(arena.params, arena.offsets)}
        self._sent = []   # (start, end) arena ranges already launched this step
        self._works = []
        self._attached = False
        self.early_elems = 0  # elements launched from inside backward in the current step
        self.last_early_elems = 0  # ... and in the last completed step (diagnostics)
        self.bytes_reduced = 0     # bytes all-reduced since the last reset_stats()
        self._exposed = []         # (start, end) device events around the post-backward wait (timing on)
        self.timing = False
        self._pending_ag = []      # rs_ag without a fused average: (work, slice, shard) awaiting scale + gather
        self._keep = []            # rs_ag on RCCL: shards alive until their gathers complete
        self._fallback_ranges = []  # rs_ag: buckets that went through a plain all_reduce (length % world)
        self._shards = None        # rs_ag on RCCL: one preallocated shard buffer, bucket b -> [b // N, ...)
        self._lp_sent = []         # bf16 wire: ranges whose reduced values still have to be copied back

    # -------------------------------------------------------------------- overlap with backward
    def attach(self):
        """Let the fused backward hand over final grads as soon as they exist (see module doc)."""
        if self.world_size > 1:
            from ..ops import hip_ops

            hip_ops.set_grad_ready_hook(self.notify)
            self._attached = True
        return self

    def detach(self):
        if self._attached:
            from ..ops import hip_ops

            hip_ops.set_grad_ready_hook(None)
            self._attached = False

    def _wire(self):
        """the tensor the collectives run on: the arena grads (fp32) or the bf16 wire copy"""
        g = self.arena.grad
        if self.grad_dtype != "bf16":
            return g
        if self._lowp is None:
            self._lowp = torch.empty(g.numel(), dtype=torch.bfloat16, device=g.device)
        return self._lowp

    def _launch(self, s: int, e: int):
        g = self._wire()
        if self.grad_dtype == "bf16":
            g[s:e].copy_(self.arena.grad[s:e])   # cast the final range onto the wire (compute stream)
            self._lp_sent.append((s, e))
        for b in range(s, e, self.bucket_elems):
            sl = g[b:min(e, b + self.bucket_elems)]
            if self.algo == "rs_ag" and sl.numel() % self.world_size == 0:
                self._launch_rs_ag(sl, b)
            else:
                if self.algo == "rs_ag":
                    self._fallback_ranges.append((b, b + sl.numel()))
                self._works.append(dist.all_reduce(sl, group=self.group, async_op=True))
        self._sent.append((s, e))

    def _launch_rs_ag(self, sl: torch.Tensor, b: int = 0):
        """Reduce-scatter the bucket into this rank's shard, then all-gather the reduced shards back into
        the bucket. On RCCL both are queued at once (one communicator stream orders them) and the 1/N
        average rides in the reduce-scatter (ReduceOp.AVG); elsewhere the gather waits for the reduction.
        Shards come from one preallocated buffer: the bucket starting at arena element ``b`` (length a
        multiple of N) owns ``[b // N, b // N + len / N)``, disjoint from every other bucket's."""
        n = sl.numel() // self.world_size
        nccl = sl.is_cuda and dist.get_backend(self.group) == "nccl"
        if nccl:
            if self._shards is None or self._shards.dtype != sl.dtype:
                self._shards = torch.empty(self.arena.numel // self.world_size + 1, dtype=sl.dtype, device=sl.device)
            shard = self._shards[b // self.world_size:b // self.world_size + n]
        else:
            shard = torch.empty(n, dtype=sl.dtype, device=sl.device)
        avg = self.average and nccl
        w = dist.reduce_scatter_tensor(shard, sl, op=dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM, group=self.group,
                                       async_op=True)
        if nccl:
            self._works.append(w)
            self._works.append(dist.all_gather_into_tensor(sl, shard, group=self.group, async_op=True))
        else:
            self._pending_ag.append((w, sl, shard))

    def _finish_rs_ag(self):
        for w, sl, shard in self._pending_ag:
            w.wait()
            if self.average:
                shard.mul_(1.0 / self.world_size)
            self._works.append(dist.all_gather_into_tensor(sl, shard, group=self.group, async_op=True))
        self._pending_ag = []

    @torch.no_grad()
    def bucket_busbw(self, reps: int = 3):
        """Every bucket's collective alone under the configured algorithm (the arena grads are restored
        afterwards): ``[{"mb", "ms", "busbw_GBps"}]``, bus bandwidth as nccl-tests reports it."""
        import time

        g = self.arena.grad
        saved = g.clone()
        out = []
        sync = torch.cuda.synchronize if g.is_cuda else (lambda: None)
        for s, e in self.buckets:
            sync()
            dist.barrier(group=self.group)
            t0 = time.perf_counter()
            for _ in range(reps):
                self._launch(s, e)
                self._finish_rs_ag()
                for w in self._works:
                    w.wait()
                self._works, self._sent, self._keep, self._fallback_ranges, self._lp_sent = [], [], [], [], []
            sync()
            t = (time.perf_counter() - t0) / reps
            ts = [None] * self.world_size
            dist.all_gather_object(ts, t, group=self.group)
            t = max(ts)
            nbytes = (e - s) * g.element_size()
            out.append({"mb": round(nbytes / 2 ** 20, 1), "ms": round(t * 1e3, 3),
                        "busbw_GBps": round(2 * (self.world_size - 1) / self.world_size * nbytes / t / 1e9, 1)})
        g.copy_(saved)
        return out

    @torch.no_grad()
    def notify(self, params):
        """All-reduce the arena ranges of ``params`` now (their grads are final for this step)."""
        if self.world_size <= 1:
            return
        rs = sorted(self._range[id(p)] for p in params if id(p) in self._range)
        for o, n in rs:
            if any(o < e and s < o + n for s, e in self._sent):
                # a second hooked backward before all_reduce(): its grads would be summed across peers
                # twice and accumulate into buffers whose collective is still in flight
                raise RuntimeError("GradSync: a gradient range was handed over twice in one step -- one backward() "
                                   "per all_reduce() while attached (disable the overlap for gradient accumulation)")
        merged = []
        for o, n in rs:
            if merged and o <= merged[-1][1]:
                merged[-1][1] = max(merged[-1][1], o + n)
            else:
                merged.append([o, o + n])
        for s, e in merged:
            self._launch(s, e)
            self.early_elems += e - s

    def _remaining(self):
        out, cur = [], 0
        for s, e in sorted(self._sent):
            if s > cur:
                out.append((cur, s))
            cur = max(cur, e)
        if cur < self.arena.numel:
            out.append((cur, self.arena.numel))
        return out

    def reset_stats(self):
        self.bytes_reduced = 0
        self._exposed = []

    def exposed_ms(self) -> float:
        """Device time the compute stream spent between the end of backward and the completion of the
        step's gradient all-reduce (the part NOT hidden under backward), summed since reset_stats();
        synchronises the events."""
        tot = 0.0
        for a, b in self._exposed:
            b.synchronize()
            tot += a.elapsed_time(b)
        return tot

    @torch.no_grad()
    def all_reduce(self):
        if self.world_size <= 1:
            return
        g = self.arena.grad
        ev0 = None
        if self.timing and g.is_cuda:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        self.bytes_reduced += g.numel() * (2 if self.grad_dtype == "bf16" else 4)
        for s, e in self._remaining():
            self._launch(s, e)
        self._finish_rs_ag()
        for w in self._works:
            w.wait()
        self._works, self._sent, self._keep = [], [], []
        if self.grad_dtype == "bf16":
            lp = self._lowp
            for s, e in self._lp_sent:
                g[s:e].copy_(lp[s:e])
            self._lp_sent = []
        self.last_early_elems, self.early_elems = self.early_elems, 0
        if ev0 is not None:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record()
            self._exposed.append((ev0, ev1))
        if self.average:
            if self.algo == "rs_ag":
                # buckets that went through rs_ag are averaged already; all_reduce fallbacks (a bucket whose
                # length is not a multiple of the world) still need the scale
                self._scale_fallbacks(g)
            else:
                g.mul_(1.0 / self.world_size)

    def _scale_fallbacks(self, g):
        for b0, b1 in self._fallback_ranges:
            g[b0:b1].mul_(1.0 / self.world_size)
        self._fallback_ranges = []


@torch.no_grad()
def tune_grad_sync(arena: FlatArena, world_size: int, group=None, grad_dtype: str = "fp32",
                   algos=("rccl", "rs_ag"), bucket_mb=(16, 32, 64, 128), reps: int = 3, step_fn=None,
                   overlap: bool = True, top: int = 3, step_reps: int = 2):
    """Time the full-arena gradient all-reduce for every (algorithm, bucket size) candidate on the real
    communicator and return ``(algo, bucket_bytes, table)`` of the fastest. Times are the max over ranks
    (``all_gather_object``), so every rank sees the same table and selects the same candidate. The arena
    grads are restored afterwards. With one rank there is nothing to tune: the defaults come back.

    ``step_fn(gs)``: a training step body (zero grads, forward, backward, ``gs.all_reduce()``) -- the
    ``top`` standalone winners are then re-timed INSIDE it, with the candidate attached to the fused
    backward (``overlap``), and the selection is made on that ``step_ms`` column: in the step most of the
    bytes leave during backward, beside MFMA-heavy kernels, where the standalone order need not hold."""
    import time

    if world_size <= 1:
        return "rccl", DEFAULT_BUCKET_BYTES, []
    g = arena.grad
    saved = g.clone()
    sync = torch.cuda.synchronize if g.is_cuda else (lambda: None)

    def timed(fn, n):
        sync()
        dist.barrier(group=group)
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        sync()
        t = (time.perf_counter() - t0) / n
        ts = [None] * world_size
        dist.all_gather_object(ts, t, group=group)
        return max(ts)

    table = []
    for algo in algos:
        for mb in bucket_mb:
            gs = GradSync(arena, world_size=world_size, group=group, grad_dtype=grad_dtype,
                          bucket_bytes=int(mb * 2 ** 20), algo=algo)
            gs.all_reduce()          # warm-up: communicator paths, shard / wire buffers
            t = timed(gs.all_reduce, reps)
            nbytes = g.numel() * (2 if grad_dtype == "bf16" else 4)
            table.append({"algo": algo, "bucket_mb": mb, "ms": round(t * 1e3, 3),
                          "busbw_GBps": round(2 * (world_size - 1) / world_size * nbytes / t / 1e9, 1),
                          "step_ms": None})
            g.copy_(saved)
    key = "ms"
    if step_fn is not None and len(table) > 1:
        for row in sorted(table, key=lambda r: (r["ms"], r["algo"], r["bucket_mb"]))[:top]:
            gs = GradSync(arena, world_size=world_size, group=group, grad_dtype=grad_dtype,
                          bucket_bytes=int(row["bucket_mb"] * 2 ** 20), algo=row["algo"])
            if overlap:
                gs.attach()
            try:
                with torch.enable_grad():
                    step_fn(gs)      # warm-up of this candidate inside the step
                    row["step_ms"] = round(timed(lambda: step_fn(gs), step_reps) * 1e3, 3)
            finally:
                gs.detach()
        key = "step_ms"
    g.copy_(saved)
    del saved
    ranked = [r for r in table if r[key] is not None]
    best = min(ranked, key=lambda r: (r[key], r["algo"], r["bucket_mb"]))
    return best["algo"], int(best["bucket_mb"] * 2 ** 20), table
