set -o pipefail
# fused reversible stack: numerics tests, then the reference recipe + 1.3B config throughput
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_model_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rev.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_rev.log; exit 1; }
tail -2 gpurun_out/pytest_rev.log
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python3 bench.py "$@" --profile-steps 2 > gpurun_out/cfg_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/cfg_$name.log; exit 1; }
  grep -h "metric\|phase" gpurun_out/cfg_$name.log | cut -c1-120,400-900
}
run ref16 300 --model reference --batch 16 --steps 3 --warmup 1
run ref48 300 --model reference --batch 48 --steps 3 --warmup 1
run l13_32 300 --model dalle-1.3b --batch 32 --steps 3 --warmup 1
