# attention kernel check: GPU numerics tests of the attention kernels + standalone forward / backward timings
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-attn}
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for d in 0 4 8 16 35 39 7; do
  DALLE_AMD_ATTN_DIAG=$d timeout -k 10 120 python3 benchmarks/attn_fwd_diag.py || exit 1
done
