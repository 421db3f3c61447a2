set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DALLE_AMD_ATTN_OCC=3,3,3,3 timeout -k 10 200 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/pytest_occ3.log 2>&1 || { echo "occ3 tests failed"; tail -30 gpurun_out/pytest_occ3.log; exit 1; }
tail -1 gpurun_out/pytest_occ3.log
for occ in 2,2,2,2 3,2,2,2 3,3,3,3; do
  tag=$(echo $occ | tr , _)
  DALLE_AMD_ATTN_OCC=$occ timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/occ_$tag -o run --output-format csv -- python3 benchmarks/bench_ops.py --only attn --batch 48 > gpurun_out/occ_$tag.log 2>&1 || { echo "prof $occ failed"; tail -20 gpurun_out/occ_$tag.log; exit 1; }
  rm -f gpurun_out/occ_$tag/run_kernel_trace.csv
  echo "== $occ"; grep '"op"' gpurun_out/occ_$tag.log
  python3 scripts/prof_summary.py gpurun_out/occ_$tag/run_kernel_stats.csv 8
done
