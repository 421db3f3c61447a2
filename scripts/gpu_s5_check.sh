set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_s5b.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu_s5b.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_s5b.log
timeout -k 10 300 python3 bench.py --profile-steps 3 > gpurun_out/bench_s5b.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_s5b.log; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_s5b.log
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/attn_fused -o run --output-format csv -- python3 benchmarks/bench_ops.py --only attn --batch 48 > gpurun_out/attn_fused.log 2>&1 || { echo "prof attn failed"; tail -20 gpurun_out/attn_fused.log; exit 1; }
rm -f gpurun_out/attn_fused/run_kernel_trace.csv
grep '"op"' gpurun_out/attn_fused.log
python3 scripts/prof_summary.py gpurun_out/attn_fused/run_kernel_stats.csv 8
