"""Logging helpers mirroring ``hivemind.utils.logging`` (``run_trainer.py:9,20-21``)."""
from __future__ import annotations

import logging
import os
import sys

_FMT = "%(asctime)s.%(msecs)03d [%(levelname)s] [%(name)s.%(funcName)s:%(lineno)d] %(message)s"
_configured = False


def _configure_root(level=None):
    global _configured
    if _configured:
        return
    level = level or os.environ.get("DALLE_AMD_LOGLEVEL", "INFO")
    handler = logging.StreamHandler(sys.stderr)
    handler.setFormatter(logging.Formatter(_FMT, datefmt="%b %d %H:%M:%S"))
    root = logging.getLogger("dalle_amd")
    root.addHandler(handler)
    root.setLevel(level)
    root.propagate = False
    _configured = True


def get_logger(name: str = None) -> logging.Logger:
    _configure_root()
    if name is None:
        return logging.getLogger("dalle_amd")
    if not name.startswith("dalle_amd"):
        name = "dalle_amd." + name
    return logging.getLogger(name)


def use_hivemind_log_handler(where: str = "in_root_logger"):
    """Route the package handler into the root logger (reference calls this with 'in_root_logger')."""
    _configure_root()
    if where == "in_root_logger":
        root = logging.getLogger()
        pkg = logging.getLogger("dalle_amd")
        if pkg.handlers and not root.handlers:
            root.addHandler(pkg.handlers[0])
            root.setLevel(pkg.level)
