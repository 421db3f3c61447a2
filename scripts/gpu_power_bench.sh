#!/bin/bash
# Board power / shader clock sampled (rocm-smi, read-only) while bench.py runs its default config for 40 steps.
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --steps 40 --warmup 3 > gpurun_out/power_bench.log 2>&1 &
BP=$!
: > gpurun_out/power_bench_smi.log
while kill -0 $BP 2>/dev/null; do
  timeout 20 rocm-smi --showpower --showclocks --json >> gpurun_out/power_bench_smi.log 2>/dev/null
  echo >> gpurun_out/power_bench_smi.log
  sleep 0.3
done
wait $BP
