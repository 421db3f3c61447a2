# text dK/dV two-tile software pipeline: attention tests, per-kernel profile of the parts bench, bench step
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pipe_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pipe_tests.log; exit 1; }
tail -1 gpurun_out/pipe_tests.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/pipeprof -o run -- python3 benchmarks/bench_attn_parts.py 128 > gpurun_out/pipeprof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/pipeprof.log; exit 1; }
grep bench24 gpurun_out/pipeprof.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/pipe_bench_$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/pipe_bench_$i.log; exit 1; }
  echo "bench $(grep '^{' gpurun_out/pipe_bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
