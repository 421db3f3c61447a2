set -o pipefail
# BASELINE configs 3 and 4 + the reference 64-layer recipe on one MI355X
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python3 bench.py "$@" --profile-steps 2 > gpurun_out/cfg_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/cfg_$name.log; exit 1; }
  grep -h "metric\|phase" gpurun_out/cfg_$name.log | cut -c1-400
}
run psgd8 240 --steps 5 --warmup 2 --compression powersgd --optim-bits 8
run ref 300 --model reference --batch 16 --steps 3 --warmup 1
run l13 300 --model dalle-1.3b --batch 16 --steps 3 --warmup 1
