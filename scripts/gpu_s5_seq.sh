set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -q --timeout 150 --timeout-method thread > gpurun_out/pytest_seq.log 2>&1 || { echo "pytest failed"; tail -50 gpurun_out/pytest_seq.log; exit 1; }
tail -1 gpurun_out/pytest_seq.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_seq -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_seq.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_seq.log; exit 1; }
rm -f gpurun_out/prof_seq/run_kernel_trace.csv
python3 scripts/prof_summary.py gpurun_out/prof_seq/run_kernel_stats.csv 16 7
timeout -k 10 300 python3 bench.py --profile-steps 3 > gpurun_out/bench_seq.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_seq.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_seq.log | cut -c1-300
DALLE_AMD_FUSED_SEQUENTIAL=0 timeout -k 10 300 python3 bench.py > gpurun_out/bench_seq0.log 2>&1 || { echo "bench0 failed"; tail -20 gpurun_out/bench_seq0.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_seq0.log | cut -c1-200
