# attention schedule variants: tests + fwd+bwd timing + kernel breakdown
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DALLE_AMD_ATTN_ORDER=${ORDER:-4} timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/attnv_test.log 2>&1 || { echo "attention tests failed"; tail -40 gpurun_out/attnv_test.log; exit 1; }
tail -1 gpurun_out/attnv_test.log
timeout -k 10 300 python3 -u benchmarks/bench_attn_variants.py 64 ${VARIANTS:-0,4} > gpurun_out/attnv.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/attnv.log; exit 1; }
grep -v amdgpu.ids gpurun_out/attnv.log
for o in 0 ${ORDER:-4}; do
  DALLE_AMD_ATTN_ORDER=$o timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/attnv_prof$o -o run --output-format csv -- python3 benchmarks/bench_attn_kernel.py axial_row 64 5 > gpurun_out/attnv_prof$o.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/attnv_prof$o.log; exit 1; }
  echo "order $o:"; python3 scripts/prof_summary.py gpurun_out/attnv_prof$o/run_kernel_stats.csv 6 1 | tail -5
done
