set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_dq.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_dq.log; exit 1; }
tail -1 gpurun_out/pytest_dq.log
for occ in 3,3,2,2 2,3,2,2; do
  tag=$(echo $occ | tr , _)
  DALLE_AMD_ATTN_OCC=$occ timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/dq_$tag -o run --output-format csv -- python3 benchmarks/bench_ops.py --only attn --batch 48 > gpurun_out/dq_$tag.log 2>&1 || { echo "prof $occ failed"; tail -20 gpurun_out/dq_$tag.log; exit 1; }
  rm -f gpurun_out/dq_$tag/run_kernel_trace.csv
  echo "== $occ"; grep '"op"' gpurun_out/dq_$tag.log
  python3 scripts/prof_summary.py gpurun_out/dq_$tag/run_kernel_stats.csv 6
done
timeout -k 10 300 python3 bench.py > gpurun_out/bench_dq.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_dq.log; exit 1; }
grep '^{' gpurun_out/bench_dq.log | cut -c1-200
