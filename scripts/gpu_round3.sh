set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python benchmarks/bench_ops.py > gpurun_out/bench_ops.log 2>&1 || { echo "ops bench failed"; tail -30 gpurun_out/bench_ops.log; exit 1; }
cat gpurun_out/bench_ops.log | grep op
for B in 16 32; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --batch $B > gpurun_out/bench_hip_b$B.log 2>&1 || { echo "bench B=$B failed"; tail -20 gpurun_out/bench_hip_b$B.log; exit 1; }
  tail -1 gpurun_out/bench_hip_b$B.log
done
timeout -k 10 400 python benchmarks/bench_inference.py --batch 8 --iters 1 --model bench24 > gpurun_out/bench_inf_small.log 2>gpurun_out/bench_inf_small.err || { echo "inference bench failed"; tail -30 gpurun_out/bench_inf_small.err; exit 1; }
cat gpurun_out/bench_inf_small.err; tail -1 gpurun_out/bench_inf_small.log
