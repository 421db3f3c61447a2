# hipBLASLt measured-solution weight grads: tests, the per-shape survey at M = 163840, then the bench step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_blaslt_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wlt_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/wlt_tests.log; exit 1; }
tail -1 gpurun_out/wlt_tests.log
timeout -k 10 400 python3 -u benchmarks/bench_wgrad_lt.py > gpurun_out/wlt_survey.jsonl 2>&1 || { echo "survey failed"; tail -10 gpurun_out/wlt_survey.jsonl; exit 1; }
grep '^{' gpurun_out/wlt_survey.jsonl
for v in 1 0 1 0; do
  DALLE_AMD_WGRAD_LT=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/wlt_bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/wlt_bench_$v.log; exit 1; }
  echo "lt=$v $(grep '^{' gpurun_out/wlt_bench_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
