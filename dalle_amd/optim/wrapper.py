"""Delegating optimizer base (the role of the reference's dead-code ``lib/training/wrapper.py``).

``DelegatingOptimizer(inner)`` behaves as ``inner`` for everything it does not override -- the torch
``Optimizer`` protocol (``param_groups``, ``state``, ``defaults``, ``state_dict``/``load_state_dict``,
``step``, ``zero_grad``, ``add_param_group``) and any extra attribute -- so a subclass only writes the
behaviour it changes. Its subclass ``HostOffloadOptimizer`` (R14) steps any torch optimizer on pinned
host copies; the flat LAMB path offloads through ``MasterParams`` + ``AsyncStep`` (``parallel/delayed.py``)
instead.
"""
from __future__ import annotations

import torch


class DelegatingOptimizer(torch.optim.Optimizer):
    _own = ("inner",)

    def __init__(self, inner: torch.optim.Optimizer):  # noqa: D107 - torch's __init__ is deliberately skipped
        object.__setattr__(self, "inner", inner)

    def __getattr__(self, name):
        # only reached for attributes this object does not have itself
        return getattr(object.__getattribute__(self, "inner"), name)

    def __setattr__(self, name, value):
        if name in type(self)._own or name in type(self).__dict__:
            object.__setattr__(self, name, value)
        else:
            setattr(self.inner, name, value)

    # the protocol members torch.optim.Optimizer defines as real methods / properties
    param_groups = property(lambda self: self.inner.param_groups)
    state = property(lambda self: self.inner.state)
    defaults = property(lambda self: self.inner.defaults)

    def state_dict(self):
        return self.inner.state_dict()

    def load_state_dict(self, state_dict):
        return self.inner.load_state_dict(state_dict)

    def step(self, closure=None):
        return self.inner.step(closure)

    def zero_grad(self, set_to_none: bool = True):
        return self.inner.zero_grad(set_to_none=set_to_none)

    def add_param_group(self, param_group):
        return self.inner.add_param_group(param_group)

    def __repr__(self):
        return f"{type(self).__name__}({self.inner!r})"


# the reference's name
OptimizerWrapper = DelegatingOptimizer


class HostOffloadOptimizer(DelegatingOptimizer):
    """Any torch optimizer, stepping on pinned host copies of its parameters (the reference's
    ``lib/training/offload.py:10-93``) -- for optimizers this build has no fused HIP step for.

    The flat LAMB path offloads through ``MasterParams(device="cpu")`` (``parallel/delayed.py``); this wrapper
    is the generic one ``CollaborativeOptimizer`` uses when it is handed an already-built optimizer together
    with ``offload_device``. Instead of one copy per tensor, the grads (and with ``full_sync`` the params)
    are packed into one device staging vector (one ``cat`` kernel), moved with ONE D2H copy into a
    contiguous pinned buffer whose slices are the host parameters / grads, the inner step runs on the CPU,
    and ONE H2D copy plus a ``_foreach_copy_`` put the result back. The optimizer state is created on the
    host (the step sees only the host parameters). Host master and state are fp32 whatever the model dtype.
    """
    _own = ("inner", "full_sync", "_dev_params", "_host_params", "_host", "_hgrad", "_stage", "_sizes")

    def __init__(self, inner: torch.optim.Optimizer, full_sync: bool = True):
        super().__init__(inner)
        self.full_sync = full_sync
        self._dev_params = [list(g["params"]) for g in inner.param_groups]
        flat = [p for ps in self._dev_params for p in ps]
        self._sizes = [p.numel() for p in flat]
        n = sum(self._sizes)
        dev = flat[0].device if flat else torch.device("cpu")
        pin = dev.type == "cuda"
        self._host = torch.empty(n, dtype=torch.float32, pin_memory=pin)
        self._hgrad = torch.zeros(n, dtype=torch.float32, pin_memory=pin)
        self._stage = torch.empty(n, dtype=torch.float32, device=dev)
        hp, hg = self._host.split(self._sizes), self._hgrad.split(self._sizes)
        self._host_params, i = [], 0
        for ps in self._dev_params:
            group = []
            for p in ps:
                q = torch.nn.Parameter(hp[i].view_as(p), requires_grad=p.requires_grad)
                q.grad = hg[i].view_as(p)
                group.append(q)
                i += 1
            self._host_params.append(group)
        self._to_host(params=True, grads=False)

    @torch.no_grad()
    def _to_host(self, params: bool, grads: bool):
        flat = [p for ps in self._dev_params for p in ps]
        if not flat:
            return
        if params:
            torch.cat([p.detach().reshape(-1).float() for p in flat], out=self._stage)
            self._host.copy_(self._stage, non_blocking=True)
        if grads:
            torch.cat([(p.grad.reshape(-1).float() if p.grad is not None else torch.zeros(p.numel(), device=p.device))
                       for p in flat], out=self._stage)
            self._hgrad.copy_(self._stage, non_blocking=True)
        if self._stage.is_cuda:
            torch.cuda.current_stream(self._stage.device).synchronize()  # the CPU step reads the buffers

    @torch.no_grad()
    def _to_device(self):
        flat = [p for ps in self._dev_params for p in ps]
        if not flat:
            return
        self._stage.copy_(self._host, non_blocking=True)  # ordered before the next D2H on this stream
        torch._foreach_copy_([p.data for p in flat], [s.view_as(p) for s, p in zip(self._stage.split(self._sizes), flat)])

    def _swapped(self):
        inner = self
        class _Swap:
            def __enter__(self_):
                for g, hp in zip(inner.inner.param_groups, inner._host_params):
                    g["params"] = hp
            def __exit__(self_, *exc):
                for g, dp in zip(inner.inner.param_groups, inner._dev_params):
                    g["params"] = dp
        return _Swap()

    def step(self, closure=None):
        if closure is not None:
            raise ValueError("HostOffloadOptimizer does not take a closure (the step runs on host copies)")
        self._to_host(params=self.full_sync, grads=True)
        with self._swapped():
            out = self.inner.step()
        self._to_device()
        return out

    def zero_grad(self, set_to_none: bool = True):
        self.inner.zero_grad(set_to_none=set_to_none)  # the model's grads
        self._hgrad.zero_()

    def state_dict(self):
        with self._swapped():
            return self.inner.state_dict()

    def load_state_dict(self, state_dict):
        with self._swapped():  # torch casts the loaded state to the (host) parameters' device
            return self.inner.load_state_dict(state_dict)

    def add_param_group(self, param_group):
        raise NotImplementedError("HostOffloadOptimizer packs its parameters once; build a new one instead")


# the reference's name
OffloadOptimizer = HostOffloadOptimizer
