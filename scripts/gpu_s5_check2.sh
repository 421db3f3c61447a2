set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_attn2.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_attn2.log; exit 1; }
tail -2 gpurun_out/pytest_attn2.log
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/attn_fused2 -o run --output-format csv -- python3 benchmarks/bench_ops.py --only attn --batch 48 > gpurun_out/attn_fused2.log 2>&1 || { echo "prof attn failed"; tail -20 gpurun_out/attn_fused2.log; exit 1; }
rm -f gpurun_out/attn_fused2/run_kernel_trace.csv
grep '"op"' gpurun_out/attn_fused2.log
python3 scripts/prof_summary.py gpurun_out/attn_fused2/run_kernel_stats.csv 8
timeout -k 10 300 python3 bench.py --profile-steps 3 > gpurun_out/bench_s5c.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_s5c.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_s5c.log
