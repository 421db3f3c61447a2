# bench24 step with a larger hipBLASLt workspace for torch's GEMMs (HIPBLASLT_WORKSPACE_SIZE, KiB) vs the default, alternating
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in default 262144 default 262144; do
  if [ $v = default ]; then cmd="timeout -k 10 300 python3 bench.py --steps 10 --warmup 3"; else cmd="env HIPBLASLT_WORKSPACE_SIZE=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 3"; fi
  $cmd > gpurun_out/ws_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/ws_$v.log; exit 1; }
  echo "ws=$v $(grep '^{' gpurun_out/ws_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
