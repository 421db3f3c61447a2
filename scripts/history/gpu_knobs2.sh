# bench24 step at the default micro-batch under kernel launch knobs (attention occupancy / concurrency, QKV tile order)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  env $1 timeout -k 10 300 python3 bench.py --steps 15 --warmup 3 > gpurun_out/knob2.log 2>&1 || { echo "bench failed ($1)"; tail -5 gpurun_out/knob2.log; exit 1; }
  echo "$1 $(grep '^{' gpurun_out/knob2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for cfg in "X=0" "DALLE_AMD_ATTN_BWD_CONC=1" "DALLE_AMD_ATTN_OCC=2,3,2,2" "DALLE_AMD_ATTN_OCC=3,2,2,2" "DALLE_AMD_PT_GROUP=8" "DALLE_AMD_PT_GROUP=2" "DALLE_AMD_PT_GROUP=-4" "DALLE_AMD_PT_PERSIST=1" "DALLE_AMD_GEMM_NT_STORE=1" "X=0"; do
  run "$cfg"
done
