# coalesced dQ prologue + full-row rotary backward stores: attention tests, parts (new vs round-3 prologue), bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dqp_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/dqp_tests.log; exit 1; }
tail -1 gpurun_out/dqp_tests.log
for d in 0 256 0 256; do
  DALLE_AMD_ATTN_DIAG=$d timeout -k 10 120 python3 -u benchmarks/bench_attn_parts.py 128 > gpurun_out/dqp_parts_$d.log 2>&1 || { echo "parts $d failed"; tail -5 gpurun_out/dqp_parts_$d.log; exit 1; }
  echo "diag=$d $(grep -h 'bench24_attention' gpurun_out/dqp_parts_$d.log) $(grep -h axial_row gpurun_out/dqp_parts_$d.log)"
done
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/dqp_bench_$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/dqp_bench_$i.log; exit 1; }
  echo "bench $(grep '^{' gpurun_out/dqp_bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
