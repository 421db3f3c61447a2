# attention forward kernel change check: kernel numerics, standalone forward timing (with the measurement-only
# phase skips), then the bench24 step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
for d in ${DIAGS:-0 4}; do
  DALLE_AMD_ATTN_DIAG=$d timeout -k 10 120 python3 benchmarks/attn_fwd_diag.py || exit 1
done
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/attn_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/attn_bench.log; exit 1; }
grep metric gpurun_out/attn_bench.log | cut -c1-200
