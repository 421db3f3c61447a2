"""hipBLASLt / rocBLAS solution selection for the plain library GEMMs (PyTorch TunableOp).

The fused and hot non-GEMM ops are hand-written HIP kernels; the remaining plain GEMMs go to
hipBLASLt, whose heuristic pick is not always the fastest solution for our shapes (measured: FF-in
forward M=20480 N=8192 K=1024 0.283 ms by heuristic vs 0.249 ms by the best solution). TunableOp
benchmarks the candidate solutions once per shape and records the winners in a CSV keyed by GPU
arch / ROCm / hipBLASLt versions (the validators: a file from another stack is ignored).

* ``tune``: search and record (``--tunable tune``; done once per machine image, off the timed path);
* ``use`` : load the recorded winners, no searching (the default when the file exists);
* ``off`` : library heuristics only.
"""
from __future__ import annotations

import os

DEFAULT_FILE = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "profiles",
                            "tunableop_gfx950.csv")


def setup_gemm_tuning(mode: str = "auto", path: str = DEFAULT_FILE) -> str:
    import torch

    if not torch.cuda.is_available() or mode == "off":
        return "off"
    import torch.cuda.tunable as tun

    if mode == "auto":
        mode = "use" if os.path.exists(path) else "off"
        if mode == "off":
            return mode
    tun.enable(True)
    if mode == "tune":
        tun.tuning_enable(True)
        tun.set_max_tuning_iterations(50)
        tun.set_filename(path, insert_device_ordinal=False)
    else:
        tun.tuning_enable(False)
        tun.read_file(path)
    return mode
