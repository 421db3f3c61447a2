set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_delayed_gpu.py tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -k "delayed or random_geometry" > gpurun_out/pytest_new_s5.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_new_s5.log; exit 1; }
tail -8 gpurun_out/pytest_new_s5.log
