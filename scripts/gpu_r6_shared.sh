# round 6: decode with one caption repeated over the batch (the reference's run_inference workload): text keys read
# from row 0's cache. Exactness tests, then images/s distinct vs repeated captions, then the repeated-caption trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_generation_gpu.py tests/test_skinny_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6s_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6s_tests.log | head -30; tail -30 gpurun_out/r6s_tests.log; exit 1; }
tail -2 gpurun_out/r6s_tests.log
for c in "" --same-caption "" --same-caption; do
  timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --iters 2 $c > gpurun_out/r6s_inf.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r6s_inf.log; exit 1; }
  echo "caption=${c:-distinct} $(grep -h '^{' gpurun_out/r6s_inf.log | cut -c1-330)"
done
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dec7 -o run --output-format csv -- python3 $R/benchmarks/bench_inference.py --batch 64 --model reference --profile-steps 32 --no-vae --same-caption > $R/gpurun_out/prof_dec7.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_dec7.log; exit 1; }
cd $R
python3 scripts/decode_trace_summary.py gpurun_out/prof_dec7/run_kernel_trace.csv --steps 16 > gpurun_out/r6s_trace_summary.txt
rm -f gpurun_out/prof_dec7/run_kernel_trace.csv
head -24 gpurun_out/r6s_trace_summary.txt
