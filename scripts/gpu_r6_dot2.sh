# round 6: decode attention with packed-bf16 dot products (v_dot2c_f32_bf16: q.k without unpacking, P.V two keys per
# instruction): decode tests, then images/s distinct / repeated captions, then the kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_generation_gpu.py tests/test_skinny_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6t_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6t_tests.log | head -30; tail -30 gpurun_out/r6t_tests.log; exit 1; }
tail -2 gpurun_out/r6t_tests.log
for c in "" --same-caption "" --same-caption; do
  timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --iters 2 $c > gpurun_out/r6t_inf.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r6t_inf.log; exit 1; }
  echo "caption=${c:-distinct} $(grep -h '^{' gpurun_out/r6t_inf.log | cut -c1-330)"
done
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dec8 -o run --output-format csv -- python3 $R/benchmarks/bench_inference.py --batch 64 --model reference --profile-steps 32 --no-vae > $R/gpurun_out/prof_dec8.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_dec8.log; exit 1; }
cd $R
python3 scripts/decode_trace_summary.py gpurun_out/prof_dec8/run_kernel_trace.csv --steps 16 > gpurun_out/r6t_trace_summary.txt
rm -f gpurun_out/prof_dec8/run_kernel_trace.csv
grep -A 8 "us/step  calls" gpurun_out/r6t_trace_summary.txt; head -3 gpurun_out/r6t_trace_summary.txt
