# round 6, final tree: generation (distinct / repeated caption, 6 batches each) and the training bench, one box
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for cap in "" "--same-caption"; do
  timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --iters 6 $cap > gpurun_out/r6f_gen.log 2>&1 || { echo "gen $cap failed"; tail -5 gpurun_out/r6f_gen.log; exit 1; }
  echo "gen cap=${cap:-distinct} $(grep -E '^# (generate|batched)' gpurun_out/r6f_gen.log | tr '\n' ' ')"
  grep '^{' gpurun_out/r6f_gen.log | cut -c1-700
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6f_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r6f_bench.log; exit 1; }
grep '^{' gpurun_out/r6f_bench.log | cut -c1-400
