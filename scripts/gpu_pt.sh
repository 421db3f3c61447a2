# persistent GEMM family: correctness tests + interleaved benchmark vs hipBLASLt / 8-phase
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gemm_pt_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_test.log 2>&1 || { echo "pt tests failed"; tail -60 gpurun_out/pt_test.log; exit 1; }
tail -3 gpurun_out/pt_test.log
PT_GROUPS=${PT_GROUPS:-0,2,8,-4} timeout -k 10 400 python3 benchmarks/bench_gemm_pt.py > gpurun_out/pt_bench.log 2>&1 || { echo "pt bench failed"; tail -20 gpurun_out/pt_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/pt_bench.log
