set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_geglu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_geglu.log; exit 1; }
tail -2 gpurun_out/pytest_geglu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_s5b -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_s5b.log 2>&1 || { echo "rocprof train failed"; tail -20 gpurun_out/prof_s5b.log; exit 1; }
rm -f gpurun_out/prof_s5b/run_kernel_trace.csv
python3 scripts/prof_summary.py gpurun_out/prof_s5b/run_kernel_stats.csv 16 7
timeout -k 10 300 python3 bench.py --profile-steps 3 > gpurun_out/bench_s5d.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_s5d.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_s5d.log
