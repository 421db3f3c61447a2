# round 6: the one-workgroup-per-head fused attention backward -- numerics first, then device times (fused / two-kernel)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused_one_workgroup or fused_rotary or sparse_attention or axial_local" > gpurun_out/r6_attn_tests.log 2>&1 || { echo "tests failed"; grep -E "Error|assert|FAIL" gpurun_out/r6_attn_tests.log | head -30; tail -40 gpurun_out/r6_attn_tests.log; exit 1; }
tail -2 gpurun_out/r6_attn_tests.log
DALLE_AMD_ATTN_FUSED_BWD=1 timeout -k 10 200 python3 benchmarks/bench_attn_parts.py 128 > gpurun_out/r6_attn_parts_fused.log 2>&1 || { echo "bench fused failed"; tail -20 gpurun_out/r6_attn_parts_fused.log; exit 1; }
DALLE_AMD_ATTN_FUSED_BWD=0 timeout -k 10 200 python3 benchmarks/bench_attn_parts.py 128 > gpurun_out/r6_attn_parts_two.log 2>&1 || { echo "bench two failed"; tail -20 gpurun_out/r6_attn_parts_two.log; exit 1; }
echo "fused:"; cat gpurun_out/r6_attn_parts_fused.log
echo "two-kernel:"; cat gpurun_out/r6_attn_parts_two.log
# the whole training step, fused backward on / off (same box, alternating)
for f in 1 0 1 0; do
  DALLE_AMD_ATTN_FUSED_BWD=$f timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6_step_fused$f.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r6_step_fused$f.log; exit 1; }
  echo "fused=$f $(grep -h '^{' gpurun_out/r6_step_fused$f.log | cut -c1-200)"
done
