set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_model_gpu.py tests/test_fused_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rev2.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_rev2.log; exit 1; }
tail -1 gpurun_out/pytest_rev2.log
for mode in "" "--no-recompute"; do
  timeout -k 10 400 python3 bench.py --model reference --batch 48 --steps 3 --warmup 1 --profile-steps 2 $mode > gpurun_out/rev_ref48$mode.log 2>&1 || { echo "ref48 $mode failed"; tail -20 gpurun_out/rev_ref48$mode.log; exit 1; }
  grep -h "metric\|phase" gpurun_out/rev_ref48$mode.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"max_mem_gb": [0-9.]*\|"reversible": "[a-z ]*"\|phase.*'
done
