set -o pipefail
# same-box A/B of an environment switch on the bench: scripts/gpu_ab.sh NAME VALUE_A VALUE_B
mkdir -p gpurun_out
name=$1; a=$2; b=$3
for rep in 1 2; do
  for v in $a $b; do
    env "$name=$v" timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 > gpurun_out/ab_${name}_$v.log 2>&1 || { echo "bench $name=$v failed"; tail -5 gpurun_out/ab_${name}_$v.log; exit 1; }
    echo "$name=$v rep$rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${name}_$v.log)"
  done
done
