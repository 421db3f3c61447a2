# bench24 step under alternative kernel-routing knobs at the default micro-batch (one box, interleaved)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  env $1 timeout -k 10 300 python3 bench.py --steps 15 --warmup 3 > gpurun_out/knob.log 2>&1 || { echo "bench failed ($1)"; tail -5 gpurun_out/knob.log; exit 1; }
  echo "$1 $(grep '^{' gpurun_out/knob.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for cfg in "X=0" "DALLE_AMD_OWN_GEMM=1" "DALLE_AMD_FUSED_FF_IN=1" "DALLE_AMD_FUSED_GEGLU_DGRAD=0" "DALLE_AMD_FUSED_QKV=1" "DALLE_AMD_GEMM_DRAIN=0" "DALLE_AMD_HEAD_CHUNK_ROWS=32768" "DALLE_AMD_WGRAD_STREAM=1" "X=0" "BENCH_BATCH=128"; do
  run "$cfg"
done
