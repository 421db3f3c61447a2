# round 6: decode with the LayerNorm folded into the residual projections' last workgroups (skinny EPI 5):
# numerics (generation tests), images/s with the tail on / off alternating on one box, then the kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_generation_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6d_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6d_tests.log | head -30; tail -30 gpurun_out/r6d_tests.log; exit 1; }
tail -2 gpurun_out/r6d_tests.log
for t in 1 0 1 0; do
  DALLE_AMD_DECODE_LN_TAIL=$t timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --iters 2 > gpurun_out/r6d_inf$t.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r6d_inf$t.log; exit 1; }
  echo "ln_tail=$t $(grep -h '^{' gpurun_out/r6d_inf$t.log | cut -c1-300)"
done
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dec6 -o run --output-format csv -- python3 $R/benchmarks/bench_inference.py --batch 64 --model reference --profile-steps 32 --no-vae > $R/gpurun_out/prof_dec6.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_dec6.log; exit 1; }
cd $R
python3 scripts/decode_trace_summary.py gpurun_out/prof_dec6/run_kernel_trace.csv --steps 16 > gpurun_out/r6d_trace_summary.txt
rm -f gpurun_out/prof_dec6/run_kernel_trace.csv
head -30 gpurun_out/r6d_trace_summary.txt
