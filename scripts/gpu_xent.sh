# cross-entropy column-sum kernel after the LDS padding: numerics tests, bench, kernel time
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -v --timeout 150 --timeout-method thread -k "xent or head or reference_geometry or hip_matches" > gpurun_out/xent_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/xent_pytest.log; exit 1; }
tail -1 gpurun_out/xent_pytest.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/xent_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/xent_bench.log; exit 1; }
grep '^{' gpurun_out/xent_bench.log | cut -c1-200
bash scripts/gpu_prof_train.sh xent > /dev/null && grep -E "xent|all kernels" gpurun_out/prof_xent_top.txt
