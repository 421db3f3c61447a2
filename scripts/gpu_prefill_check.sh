# fused-rotary prefill: generation GPU tests, prefill time, end-to-end inference
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_generation_gpu.py > gpurun_out/pf_tests.log 2>&1 || { tail -40 gpurun_out/pf_tests.log; exit 1; }
tail -1 gpurun_out/pf_tests.log
timeout -k 10 300 python3 benchmarks/bench_prefill.py 2>&1 | grep prefill_ms || exit 1
timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 2 > gpurun_out/inf_pf.log 2>&1 || { tail -20 gpurun_out/inf_pf.log; exit 1; }
grep -h '^#\|metric' gpurun_out/inf_pf.log | cut -c1-330
