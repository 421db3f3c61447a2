set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_final.log; exit 1; }
tail -1 gpurun_out/pytest_final.log
timeout -k 10 300 python3 -c "import __graft_entry__ as e; e.smoke(); print('smoke ok')" > gpurun_out/smoke_final.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench_final.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_final.log; exit 1; }
grep '^{' gpurun_out/bench_final.log | cut -c1-200
