# GPU check: GPU tests, smoke, bench (step + collab engines), 2-rank gloo rehearsal on one GPU
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r2s4z_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r2s4z_pytest.log; exit 1; }
tail -1 gpurun_out/r2s4z_pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2s4z_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r2s4z_smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/r2s4z_bench_step.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r2s4z_bench_step.log; exit 1; }
grep '^{' gpurun_out/r2s4z_bench_step.log | cut -c1-400
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --engine collab > gpurun_out/r2s4z_bench_collab.log 2>&1 || { echo "bench collab failed"; tail -20 gpurun_out/r2s4z_bench_collab.log; exit 1; }
grep '^{' gpurun_out/r2s4z_bench_collab.log | cut -c1-400
BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --batch 8 > gpurun_out/r2s4z_bench_2rank_gloo.log 2>&1 || { echo "2-rank failed"; tail -20 gpurun_out/r2s4z_bench_2rank_gloo.log; exit 1; }
grep '^{' gpurun_out/r2s4z_bench_2rank_gloo.log | cut -c1-600
