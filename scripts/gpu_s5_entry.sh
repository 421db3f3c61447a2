set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_entrypoints_gpu.py tests/test_delayed_gpu.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_entry_gpu.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_entry_gpu.log; exit 1; }
tail -6 gpurun_out/pytest_entry_gpu.log
