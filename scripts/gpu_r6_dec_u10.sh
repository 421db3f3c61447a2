set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_generation_gpu.py tests/test_skinny_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6u_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6u_tests.log | head -30; tail -30 gpurun_out/r6u_tests.log; exit 1; }
tail -1 gpurun_out/r6u_tests.log
bash scripts/gpu_r6_shared_rerun.sh
