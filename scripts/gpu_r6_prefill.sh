# round 6: repeated-caption prefill of row 0 only -- generation tests, then images/s (and the prefill time) distinct /
# repeated captions, alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_generation_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r6p_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6p_tests.log | head -30; tail -30 gpurun_out/r6p_tests.log; exit 1; }
tail -1 gpurun_out/r6p_tests.log
for c in "" --same-caption "" --same-caption; do
  timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --iters 3 $c > gpurun_out/r6p_inf.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r6p_inf.log; exit 1; }
  echo "caption=${c:-distinct} $(grep -h '^{' gpurun_out/r6p_inf.log | grep -o '"value": [0-9.]*\|"seconds_per_batch": [0-9.]*\|"sampling_seconds": [0-9.]*\|"text_shared": \[[0-9, ]*\]' | tr '\n' ' ') $(grep -h 'batched prefill' gpurun_out/r6p_inf.log)"
done
