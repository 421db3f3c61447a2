set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 benchmarks/bench_gemm.py > gpurun_out/gemm_ours.log 2>&1 || { echo "gemm bench failed"; tail -20 gpurun_out/gemm_ours.log; exit 1; }
cat gpurun_out/gemm_ours.log | grep -v amdgpu.ids
