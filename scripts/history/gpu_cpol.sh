# GEMM output-store cache policy A/B (benchmarks/bench_gemm_cpol.py) + GEMM correctness tests + 1-GPU bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_pt_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/cpol_test.log 2>&1 || { echo "gemm tests failed"; tail -40 gpurun_out/cpol_test.log; exit 1; }
tail -1 gpurun_out/cpol_test.log
timeout -k 10 500 python3 -u benchmarks/bench_gemm_cpol.py > gpurun_out/cpol_bench.log 2>&1 || { echo "cpol bench failed"; tail -30 gpurun_out/cpol_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/cpol_bench.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > gpurun_out/cpol_bench_step.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/cpol_bench_step.log; exit 1; }
grep '^{' gpurun_out/cpol_bench_step.log | cut -c1-200
DALLE_AMD_GEMM_CPOL=17 timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > gpurun_out/cpol_bench_step17.log 2>&1 || { echo "bench17 failed"; tail -20 gpurun_out/cpol_bench_step17.log; exit 1; }
grep '^{' gpurun_out/cpol_bench_step17.log | cut -c1-200
