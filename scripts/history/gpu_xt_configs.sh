set -o pipefail
# same-box A/B of the token-contiguous weight-grad inputs (DALLE_AMD_WGRAD_XT) on the large BASELINE configs
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, xt, timeout, args...
  local name=$1 xt=$2 t=$3; shift 3
  DALLE_AMD_WGRAD_XT=$xt timeout -k 10 "$t" python3 bench.py "$@" > gpurun_out/xtcfg_${name}_$xt.log 2>&1 || { echo "$name xt=$xt failed"; tail -30 gpurun_out/xtcfg_${name}_$xt.log; exit 1; }
  echo "$name xt=$xt $(grep -h '^{' gpurun_out/xtcfg_${name}_$xt.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('max_mem_gb'), d['config'].get('per_gpu_batch'))")"
}
run ref48_auto 0 400 --model reference --batch 48 --steps 3 --warmup 1 --recompute auto
run ref48_auto 1 400 --model reference --batch 48 --steps 3 --warmup 1 --recompute auto
run l13_32_auto 0 400 --model dalle-1.3b --batch 32 --steps 3 --warmup 1 --recompute auto
run l13_32_auto 1 400 --model dalle-1.3b --batch 32 --steps 3 --warmup 1 --recompute auto
run step48 0 240 --steps 10 --warmup 3 --batch 48
run step48 1 240 --steps 10 --warmup 3 --batch 48
