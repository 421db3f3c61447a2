# non-temporal epilogue stores in the fused GEMMs: numerics, kernel times and the full step, same box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_fused_gpu.py > gpurun_out/nt_tests.log 2>&1 || { tail -30 gpurun_out/nt_tests.log; exit 1; }
tail -1 gpurun_out/nt_tests.log
for v in 0 1 0 1; do
  DALLE_AMD_GEMM_NT_STORE=$v timeout -k 10 120 python3 benchmarks/bench_fused_gemm.py 2>/dev/null | grep '^{' | sed "s/^/nt=$v /" || exit 1
done
bash scripts/gpu_ab.sh DALLE_AMD_GEMM_NT_STORE 0 1
