#!/bin/bash
# register-resident cross-entropy kernel: numerics tests, per-chunk timing vs the LDS-accumulator form
# (DALLE_AMD_XENT_REG=0), bench step A/B; grid-barrier probe (two-level form)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -v --timeout 150 --timeout-method thread -k "xent or head or reference_geometry or hip_matches" > gpurun_out/xent_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/xent_pytest.log; exit 1; }
tail -1 gpurun_out/xent_pytest.log
for f in 1 0; do
  DALLE_AMD_XENT_REG=$f timeout -k 10 120 python3 -u benchmarks/bench_xent.py > gpurun_out/xent_chunks_$f.txt 2>&1 || { cat gpurun_out/xent_chunks_$f.txt; exit 1; }
  echo "form_reg=$f"; grep '^{' gpurun_out/xent_chunks_$f.txt
done
for f in 1 0 1 0; do
  DALLE_AMD_XENT_REG=$f timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/xent_bench_$f.log 2>&1 || { tail -20 gpurun_out/xent_bench_$f.log; exit 1; }
  echo "form_reg=$f $(grep '^{' gpurun_out/xent_bench_$f.log | cut -c1-120)"
done
timeout -k 10 90 benchmarks/grid_barrier_probe > gpurun_out/grid_barrier2.txt 2>&1 || exit 1
grep two_level gpurun_out/grid_barrier2.txt
