"""Delegating optimizer base (the role of the reference's dead-code ``lib/training/wrapper.py``).

``DelegatingOptimizer(inner)`` behaves as ``inner`` for everything it does not override -- the torch
``Optimizer`` protocol (``param_groups``, ``state``, ``defaults``, ``state_dict``/``load_state_dict``,
``step``, ``zero_grad``, ``add_param_group``) and any extra attribute -- so a subclass only writes the
behaviour it changes. In this build the host-offloaded optimizer is ``MasterParams`` + ``AsyncStep``
(``parallel/delayed.py``), so nothing here re-implements offloading.
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
