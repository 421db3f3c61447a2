"""Strict checkpoint loading with an explicit allow-list (reference ``inference/run_inference.py:119``
loads strictly)."""
from __future__ import annotations

from typing import Iterable, Mapping

import torch

# buffers that are a deterministic function of the config (recomputed at construction), so an external
# checkpoint may legitimately lack them
DERIVED_BUFFERS = ("pos_emb",)


def load_state_dict_checked(module: torch.nn.Module, state_dict: Mapping[str, torch.Tensor],
                            allowed_missing: Iterable[str] = DERIVED_BUFFERS):
    """``module.load_state_dict`` that fails on ANY unexpected key and on missing keys other than those
    whose last component is in ``allowed_missing``. Returns the (tolerated) missing keys."""
    allowed = tuple(allowed_missing)
    res = module.load_state_dict(state_dict, strict=False)
    missing = [k for k in res.missing_keys if k.rsplit(".", 1)[-1] not in allowed]
    if missing or res.unexpected_keys:
        raise RuntimeError(f"checkpoint does not match the model: {len(missing)} missing keys {missing[:8]}, "
                           f"{len(res.unexpected_keys)} unexpected keys {list(res.unexpected_keys)[:8]}")
    return list(res.missing_keys)
