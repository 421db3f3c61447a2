# round 6: top-k threshold by bitwise block counts (no LDS atomics) in the fused sampler: tests, sampler kernel time,
# decode step and images/s
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_sampler_gpu.py tests/test_generation_gpu.py tests/test_serve_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6sm_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r6sm_pytest.log | head -30; tail -30 gpurun_out/r6sm_pytest.log; exit 1; }
tail -1 gpurun_out/r6sm_pytest.log
timeout -k 10 200 python3 benchmarks/bench_sampler.py > gpurun_out/r6sm_bench.log 2>&1 || { echo "sampler bench failed"; tail -5 gpurun_out/r6sm_bench.log; exit 1; }
grep '^{' gpurun_out/r6sm_bench.log
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_sm -o run --output-format csv -- python3 $R/benchmarks/bench_inference.py --batch 64 --model reference --profile-steps 16 --no-vae --same-caption > $R/gpurun_out/prof_sm.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_sm.log; exit 1; }
cd $R
grep -h "sample_kernel" gpurun_out/prof_sm/run_kernel_stats.csv | cut -d, -f1-5
rm -f gpurun_out/prof_sm/run_kernel_trace.csv
for rep in 1 2; do
  for cap in "--same-caption" ""; do
    timeout -k 10 300 python3 benchmarks/bench_inference.py --batch 64 --iters 4 $cap > gpurun_out/r6sm_gen.log 2>&1 || { echo "gen $cap failed"; tail -5 gpurun_out/r6sm_gen.log; exit 1; }
    echo "gen cap=${cap:-distinct} $(grep -E '^# batched' gpurun_out/r6sm_gen.log | tr '\n' ' ') $(grep '^{' gpurun_out/r6sm_gen.log | grep -oE '"value": [0-9.]+|"ms_per_decode_step": [0-9.]+|"sampling_seconds": [0-9.]+' | tr '\n' ' ')"
  done
done
