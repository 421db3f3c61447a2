#!/bin/bash
# MFMA energy probe (benchmarks/mfma_power.hip, built in-tree as benchmarks/mfma_power) under a rocm-smi sampler (read-only).
mkdir -p gpurun_out
timeout -k 10 120 ./benchmarks/mfma_power 5 > gpurun_out/mfma_power.log 2>&1 &
BP=$!
: > gpurun_out/mfma_power_smi.log
while kill -0 $BP 2>/dev/null; do
  echo "$(date +%s.%N) $(timeout 20 rocm-smi --showpower --showclocks --json 2>/dev/null)" >> gpurun_out/mfma_power_smi.log
  sleep 0.3
done
wait $BP
