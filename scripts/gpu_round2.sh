set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 600 python benchmarks/bench_inference.py --batch 64 --iters 1 > gpurun_out/bench_inf.log 2>&1 || { echo "inference bench failed"; tail -30 gpurun_out/bench_inf.log; exit 1; }
tail -1 gpurun_out/bench_inf.log
