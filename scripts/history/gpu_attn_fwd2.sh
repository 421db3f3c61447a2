# attention forward after a prologue / epilogue change: numerics, then standalone times (full, no work)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/attn_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -1 gpurun_out/attn_tests.log
for d in 0 0 39; do
  DALLE_AMD_ATTN_DIAG=$d timeout -k 10 120 python3 benchmarks/attn_fwd_diag.py || exit 1
done
