# round 6: the thin last text tile (T = 257: key 256 alone) on the VALU in the attention forward and dQ kernels:
# attention numerics, device times per pattern, then the whole step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6h_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6h_tests.log | head -30; tail -30 gpurun_out/r6h_tests.log; exit 1; }
tail -1 gpurun_out/r6h_tests.log
for r in 1 2; do
  timeout -k 10 200 python3 benchmarks/bench_attn_parts.py 128 > gpurun_out/r6h_parts.log 2>&1 || { echo "parts failed"; tail -20 gpurun_out/r6h_parts.log; exit 1; }
  echo "parts $(grep -h pattern gpurun_out/r6h_parts.log | tr '\n' ' ')"
done
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6h_step.log 2>&1 || { echo "step failed"; tail -20 gpurun_out/r6h_step.log; exit 1; }
  echo "step $(grep -h '^{' gpurun_out/r6h_step.log | cut -c80-200)"
done
