set -o pipefail
mkdir -p gpurun_out
for B in 8 16 32; do
  timeout -k 10 300 python bench.py --steps 6 --warmup 2 --batch $B > gpurun_out/bench_hip_b$B.log 2>&1 || { echo "bench B=$B failed"; tail -20 gpurun_out/bench_hip_b$B.log; exit 1; }
  tail -1 gpurun_out/bench_hip_b$B.log
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch 16 > gpurun_out/prof_bench.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_bench.log; exit 1; }
find gpurun_out/prof -name "*stats*" | head
