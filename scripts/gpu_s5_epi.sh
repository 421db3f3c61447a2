set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_fused_gpu.py tests/test_model_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_epi.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_epi.log; exit 1; }
tail -1 gpurun_out/pytest_epi.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_epi -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_epi.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_epi.log; exit 1; }
rm -f gpurun_out/prof_epi/run_kernel_trace.csv
python3 scripts/prof_summary.py gpurun_out/prof_epi/run_kernel_stats.csv 8 7
timeout -k 10 300 python3 bench.py > gpurun_out/bench_epi.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_epi.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_epi.log | cut -c1-200
