# decode (reference model, batch 64) under a HIP runtime environment knob set to 0 / 1, alternating, one box
# usage: bash scripts/gpu_decode_env.sh VAR   (e.g. HIP_FORCE_DEV_KERNARG, DEBUG_CLR_GRAPH_PACKET_CAPTURE)
set -o pipefail
export TMPDIR=/tmp
VAR=${1:?variable name}
mkdir -p gpurun_out
for v in 0 1 0 1; do
  env "$VAR=$v" timeout -k 10 300 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 > gpurun_out/denv_${VAR}_$v.log 2>&1 || { echo "run $v failed"; tail -20 gpurun_out/denv_${VAR}_$v.log; exit 1; }
  echo "$VAR=$v $(grep metric gpurun_out/denv_${VAR}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_decode_step"], d["seconds_per_batch"])')"
done
