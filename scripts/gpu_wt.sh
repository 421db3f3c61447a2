# transposed bf16 weight copies in one tiled kernel: bitwise test, model tests, bench, kernel profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_fused_gpu.py -x -v --timeout 150 --timeout-method thread -k "transpose_cast or reference_geometry or sequential_fused or hip_matches or geglu" > gpurun_out/wt_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/wt_pytest.log; exit 1; }
tail -1 gpurun_out/wt_pytest.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/wt_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/wt_bench.log; exit 1; }
grep '^{' gpurun_out/wt_bench.log | cut -c1-200
bash scripts/gpu_prof_train.sh wt > /dev/null && grep -E "transpose|manual_unroll|bfloat16_copy|all kernels" gpurun_out/prof_wt_top.txt
