# two bench24 step measurements back to back (noise check for small kernel changes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/bench2_$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench2_$i.log; exit 1; }
  grep -o '"value": [0-9.]*, "unit": "[a-z/]*", "n_gpus": 1, "steps": 10, "warmup": 3, "ms_per_step": [0-9.]*' gpurun_out/bench2_$i.log
done
