set -o pipefail
# same-box A/B of the per-GPU micro-batch (bench24, default engine), three alternating reps
mkdir -p gpurun_out
for rep in 1 2 3; do
  for b in 64 128; do
    steps=$(( b == 64 ? 12 : 6 ))
    timeout -k 10 300 python3 bench.py --steps $steps --warmup 3 --batch $b > gpurun_out/bab_$b.log 2>&1 || { echo "bench B$b failed"; tail -5 gpurun_out/bab_$b.log; exit 1; }
    echo "B$b rep$rep $(grep -o '"value": [0-9.]*' gpurun_out/bab_$b.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bab_$b.log)"
  done
done
