# forward attention at 4 waves/SIMD (DALLE_AMD_ATTN_OCC=4,3,2,2; 128 VGPRs with spills) vs the default 3
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
DALLE_AMD_ATTN_OCC=4,3,2,2 timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or forward" --timeout 120 --timeout-method thread > gpurun_out/occ4_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/occ4_tests.log; exit 1; }
tail -1 gpurun_out/occ4_tests.log
for o in 3,3,2,2 4,3,2,2 3,3,2,2 4,3,2,2; do
  DALLE_AMD_ATTN_OCC=$o timeout -k 10 120 python3 -u benchmarks/bench_attn_parts.py 128 > gpurun_out/occ4_$o.log 2>&1 || { echo "occ $o failed"; tail -5 gpurun_out/occ4_$o.log; exit 1; }
  echo "occ=$o $(grep -h 'bench24_attention' gpurun_out/occ4_$o.log) $(grep -h pattern gpurun_out/occ4_$o.log | tr '\n' ' ')"
done
