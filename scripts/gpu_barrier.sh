#!/bin/bash
# RCCL communicator lifecycle test + grid-barrier probe (persistent decode-layer kernel pricing)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_rccl_lifecycle_gpu.py > gpurun_out/rccl_lifecycle.log 2>&1 && \
timeout -k 10 90 benchmarks/grid_barrier_probe > gpurun_out/grid_barrier.txt 2>&1
rc=$?
tail -5 gpurun_out/rccl_lifecycle.log; cat gpurun_out/grid_barrier.txt
exit $rc
