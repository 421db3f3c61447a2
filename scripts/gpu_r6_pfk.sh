# round 6: caption prefill on the assembly GEMMs + the prefill LN / softmax / residual kernels: tests, prefill time,
# images/s (distinct / repeated caption)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_generation_gpu.py tests/test_serve_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6pk_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r6pk_pytest.log | head -30; tail -30 gpurun_out/r6pk_pytest.log; exit 1; }
tail -1 gpurun_out/r6pk_pytest.log
timeout -k 10 200 python3 benchmarks/bench_prefill.py > gpurun_out/r6pk_pf.log 2>&1 && SAME=1 timeout -k 10 200 python3 benchmarks/bench_prefill.py >> gpurun_out/r6pk_pf.log 2>&1 || { echo "prefill bench failed"; tail -5 gpurun_out/r6pk_pf.log; exit 1; }
grep '^{' gpurun_out/r6pk_pf.log
for rep in 1 2; do
  for cap in "" "--same-caption"; do
    timeout -k 10 300 python3 benchmarks/bench_inference.py --batch 64 --iters 4 $cap > gpurun_out/r6pk_gen.log 2>&1 || { echo "gen $cap failed"; tail -5 gpurun_out/r6pk_gen.log; exit 1; }
    echo "gen cap=${cap:-distinct} $(grep -E '^# (generate|batched)' gpurun_out/r6pk_gen.log | tr '\n' ' ') $(grep '^{' gpurun_out/r6pk_gen.log | grep -oE '"value": [0-9.]+|"ms_per_decode_step": [0-9.]+|"sampling_seconds": [0-9.]+' | tr '\n' ' ')"
  done
done
