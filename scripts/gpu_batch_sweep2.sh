# per-GPU micro-batch sweep of the bench24 step (tile-count / wave-quantisation check around B48)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in ${BATCHES:-48 64 80 96 48 64 80 96}; do
  BENCH_BATCH=$b timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > gpurun_out/bs_b$b.log 2>&1 || { echo "bench b$b failed"; tail -5 gpurun_out/bs_b$b.log; exit 1; }
  echo "b$b $(grep '^{' gpurun_out/bs_b$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('max_mem_gb'))")"
done
