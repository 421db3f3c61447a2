set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 benchmarks/bench_ops.py --only gemm > gpurun_out/gemm.log 2>&1 || { echo "gemm bench failed"; tail -20 gpurun_out/gemm.log; exit 1; }
cat gpurun_out/gemm.log
timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model bench24 --iters 1 > gpurun_out/inf24.log 2>&1 || { echo "inference bench24 failed"; tail -20 gpurun_out/inf24.log; exit 1; }
cat gpurun_out/inf24.log
timeout -k 10 500 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 > gpurun_out/infref.log 2>&1 || { echo "inference reference failed"; tail -20 gpurun_out/infref.log; exit 1; }
cat gpurun_out/infref.log
timeout -k 10 400 python3 benchmarks/bench_ops.py --only gemm --tunable > gpurun_out/gemm_tunable.log 2>&1 || { echo "gemm tunable failed"; tail -20 gpurun_out/gemm_tunable.log; exit 1; }
cat gpurun_out/gemm_tunable.log
