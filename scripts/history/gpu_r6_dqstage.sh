# round 6: dQ text-tile staging variants (register pairs / LDS-DMA one step ahead x 2 or 3 tiles / two steps ahead):
# exactness vs the default, device time per variant, then the whole step for the best
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "staging_variants or fused_one_workgroup or axial_local or sparse_attention" > gpurun_out/r6q_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6q_tests.log | head -30; tail -30 gpurun_out/r6q_tests.log; exit 1; }
tail -2 gpurun_out/r6q_tests.log
for st in 0 2 3 4 0 4; do
  DQ_STAGE=$st timeout -k 10 200 python3 benchmarks/bench_attn_parts.py 128 > gpurun_out/r6q_parts$st.log 2>&1 || { echo "parts failed"; tail -20 gpurun_out/r6q_parts$st.log; exit 1; }
  echo "stage=$st $(grep -h axial gpurun_out/r6q_parts$st.log | tr '\n' ' ')"
done
for st in 0 4 0 4; do
  DQ_STAGE=$st timeout -k 10 300 python3 benchmarks/step_knobs.py --steps 20 --warmup 5 > gpurun_out/r6q_step$st.log 2>&1 || { echo "step failed"; tail -20 gpurun_out/r6q_step$st.log; exit 1; }
  echo "stage=$st $(grep -h '^{' gpurun_out/r6q_step$st.log | cut -c1-160)"
done
