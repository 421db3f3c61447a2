# LN+shift backward: both column-sum reductions in one launch -- model tests, bench, kernel profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_model_gpu.py tests/test_fused_gpu.py tests/test_kernels_gpu.py -x -v --timeout 150 --timeout-method thread -k "sequential_fused or reference_geometry or hip_matches or ln_shift or reversible" > gpurun_out/colsum_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/colsum_pytest.log; exit 1; }
tail -1 gpurun_out/colsum_pytest.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/colsum_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/colsum_bench.log; exit 1; }
grep '^{' gpurun_out/colsum_bench.log | cut -c1-200
bash scripts/gpu_prof_train.sh colsum > /dev/null && grep -E "column_sum|ln_shift_bwd|all kernels" gpurun_out/prof_colsum_top.txt
