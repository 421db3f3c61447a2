# round 6: attention forward with its text-tile DMA two steps ahead (three buffers): exactness, device time on / off
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "two_ahead or sparse_attention" > gpurun_out/r6w_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6w_tests.log | head -30; tail -30 gpurun_out/r6w_tests.log; exit 1; }
tail -2 gpurun_out/r6w_tests.log
for a in 0 1 0 1; do
  FWD_AHEAD2=$a timeout -k 10 200 python3 benchmarks/bench_attn_parts.py 128 > gpurun_out/r6w_parts$a.log 2>&1 || { echo "parts failed"; tail -20 gpurun_out/r6w_parts$a.log; exit 1; }
  echo "ahead2=$a $(grep -h pattern gpurun_out/r6w_parts$a.log | tr '\n' ' ')"
done
