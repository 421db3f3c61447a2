"""Loader for the in-tree HIP extension ``dalle_amd._C`` (built by ``setup.py build_ext --inplace``)."""
from __future__ import annotations

import importlib

_EXT = None
_ERR = None


def load_extension(required: bool = False):
    global _EXT, _ERR
    if _EXT is not None:
        return _EXT
    if _ERR is None:
        try:
            _EXT = importlib.import_module("dalle_amd._C")
            return _EXT
        except ImportError as e:  # pragma: no cover - depends on build state
            _ERR = e
    if required:
        raise RuntimeError(
            "dalle_amd._C (the HIP kernel extension) is not importable; build it with "
            "`PYTORCH_ROCM_ARCH=gfx950 python setup.py build_ext --inplace` "
            f"(import error: {_ERR})"
        )
    return None


def hip_available() -> bool:
    return load_extension(required=False) is not None
