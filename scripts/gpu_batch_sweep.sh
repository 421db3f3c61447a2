set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 40 48 64 80 96; do
  BENCH_BATCH=$b timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 > gpurun_out/bench_b$b.log 2>&1 || { echo "bench b$b failed"; tail -5 gpurun_out/bench_b$b.log; exit 1; }
  tail -1 gpurun_out/bench_b$b.log | cut -c1-200
done
