# decode: one joint graph (parts joined every step) vs one graph per part on its own stream (no per-step join)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DALLE_AMD_DECODE_GRAPHS=per-part timeout -k 10 300 python3 -u -m pytest tests/test_generation_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/dg_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/dg_pytest.log; exit 1; }
tail -1 gpurun_out/dg_pytest.log
for cfg in "joint 2" "per-part 2" "per-part 4" "joint 2" "per-part 2"; do
  set -- $cfg
  DALLE_AMD_DECODE_GRAPHS=$1 DALLE_AMD_DECODE_PARTS=$2 timeout -k 10 300 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 > gpurun_out/dg_$1_$2.log 2>&1 || { echo "bench failed $cfg"; tail -5 gpurun_out/dg_$1_$2.log; exit 1; }
  echo "$1 parts=$2: $(grep -o '"value": [0-9.]*' gpurun_out/dg_$1_$2.log) $(grep -o '"seconds_per_batch": [0-9.]*' gpurun_out/dg_$1_$2.log)"
done
