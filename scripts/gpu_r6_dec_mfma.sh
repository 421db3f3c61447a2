# round 6: repeated-caption decode attention on the MFMA (decode_attn_shared_kernel): decode tests, images/s distinct /
# repeated captions, then the repeated-caption kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_generation_gpu.py tests/test_skinny_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6m_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6m_tests.log | head -30; tail -30 gpurun_out/r6m_tests.log; exit 1; }
tail -1 gpurun_out/r6m_tests.log
bash scripts/gpu_r6_shared_rerun.sh
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dec9 -o run --output-format csv -- python3 $R/benchmarks/bench_inference.py --batch 64 --model reference --profile-steps 32 --no-vae --same-caption > $R/gpurun_out/prof_dec9.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_dec9.log; exit 1; }
cd $R
python3 scripts/decode_trace_summary.py gpurun_out/prof_dec9/run_kernel_trace.csv --steps 16 > gpurun_out/r6m_trace_summary.txt
rm -f gpurun_out/prof_dec9/run_kernel_trace.csv
grep -A 8 "us/step  calls" gpurun_out/r6m_trace_summary.txt; head -3 gpurun_out/r6m_trace_summary.txt
