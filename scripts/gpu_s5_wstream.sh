set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py tests/test_entrypoints_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ws.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_ws.log; exit 1; }
tail -1 gpurun_out/pytest_ws.log
timeout -k 10 300 python3 bench.py > gpurun_out/bench_ws.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_ws.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_ws.log | cut -c1-200
DALLE_AMD_WGRAD_STREAM=0 timeout -k 10 300 python3 bench.py > gpurun_out/bench_ws0.log 2>&1 || { echo "bench0 failed"; tail -20 gpurun_out/bench_ws0.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_ws0.log | cut -c1-200
timeout -k 10 300 python3 bench.py > gpurun_out/bench_ws1.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_ws1.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_ws1.log | cut -c1-200
