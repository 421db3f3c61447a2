set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -m pytest tests/test_fused_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -q -x > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 > gpurun_out/bench48.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench48.log; exit 1; }
tail -1 gpurun_out/bench48.log | cut -c1-250
DALLE_AMD_FUSED_QKV=0 timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 > gpurun_out/bench48_nofuse.log 2>&1 || { echo "bench nofuse failed"; tail -20 gpurun_out/bench48_nofuse.log; exit 1; }
tail -1 gpurun_out/bench48_nofuse.log | cut -c1-250
