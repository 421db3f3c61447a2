# round-3 GPU check: GPU tests, smoke, bench (step + collab engines), rocprofv3 kernel stats of the step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r3}
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_step.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench_step.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_step.log | cut -c1-300
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --engine collab > gpurun_out/${TAG}_bench_collab.log 2>&1 || { echo "bench collab failed"; tail -20 gpurun_out/${TAG}_bench_collab.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_collab.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('value','ms_per_step','collab_performance_ema_samples_per_s','collab_ema_over_wall','collab_backward_overlapped_rounds')})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv
python3 scripts/prof_summary.py gpurun_out/prof_$TAG/run_kernel_stats.csv 40 ${PROF_STEPS:-7} > gpurun_out/prof_${TAG}_top.txt
head -30 gpurun_out/prof_${TAG}_top.txt
