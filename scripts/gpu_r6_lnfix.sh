# round 6: decode LayerNorm with every load in one batch, skinny GEMM bias pairs loaded branch-free: tests, decode trace
# kernel times, images/s
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_skinny_gpu.py tests/test_generation_gpu.py tests/test_serve_gpu.py tests/test_sampler_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6ln_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r6ln_pytest.log | head -30; tail -30 gpurun_out/r6ln_pytest.log; exit 1; }
tail -1 gpurun_out/r6ln_pytest.log
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ln -o run --output-format csv -- python3 $R/benchmarks/bench_inference.py --batch 64 --model reference --profile-steps 48 --no-vae --same-caption > $R/gpurun_out/prof_ln.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_ln.log; exit 1; }
cd $R
python3 scripts/decode_trace_summary.py gpurun_out/prof_ln/run_kernel_trace.csv --steps 24 --chains 2 > gpurun_out/r6ln_trace_summary.txt
rm -f gpurun_out/prof_ln/run_kernel_trace.csv
sed -n '/us\/step  calls/,$p' gpurun_out/r6ln_trace_summary.txt | head -8
for rep in 1 2; do
  for cap in "--same-caption" ""; do
    timeout -k 10 300 python3 benchmarks/bench_inference.py --batch 64 --iters 4 $cap > gpurun_out/r6ln_gen.log 2>&1 || { echo "gen $cap failed"; tail -5 gpurun_out/r6ln_gen.log; exit 1; }
    echo "gen cap=${cap:-distinct} $(grep '^{' gpurun_out/r6ln_gen.log | grep -oE '"value": [0-9.]+|"ms_per_decode_step": [0-9.]+|"sampling_seconds": [0-9.]+' | tr '\n' ' ')"
  done
done
