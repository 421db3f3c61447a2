set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for B in ${BENCH_BATCHES:-16 32}; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --batch $B > gpurun_out/bench_hip_b$B.log 2>&1 || { echo "bench B=$B failed"; tail -20 gpurun_out/bench_hip_b$B.log; exit 1; }
  tail -1 gpurun_out/bench_hip_b$B.log
done
if [ -n "$PROFILE" ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch ${PROFILE_BATCH:-16} > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_bench.log; exit 1; }
fi
