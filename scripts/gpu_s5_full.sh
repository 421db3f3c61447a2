set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu_full_s5.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu_full_s5.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_full_s5.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s5.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_s5.log; exit 1; }
tail -1 gpurun_out/smoke_s5.log
