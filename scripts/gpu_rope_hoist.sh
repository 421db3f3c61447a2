# rotary table loads hoisted in the attention-backward epilogues: attention tests, parts, bench step
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or rotary or dkdv or dq_dma or tiles" > gpurun_out/rh_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/rh_tests.log; exit 1; }
tail -1 gpurun_out/rh_tests.log
timeout -k 10 120 python3 -u benchmarks/bench_attn_parts.py 128 > gpurun_out/rh_parts.log 2>&1 || { echo "parts failed"; tail -5 gpurun_out/rh_parts.log; exit 1; }
grep '^{' gpurun_out/rh_parts.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/rh_bench_$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/rh_bench_$i.log; exit 1; }
  echo "bench $(grep '^{' gpurun_out/rh_bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
