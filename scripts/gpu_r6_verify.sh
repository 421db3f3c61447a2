# round 6: re-check of the tree after the fused backward moved to its own translation unit: full GPU suite, smoke, bench24
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r6v_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r6v_pytest.log | head -30; tail -30 gpurun_out/r6v_pytest.log; exit 1; }
tail -2 gpurun_out/r6v_pytest.log
grep -E "GRAD_ERR|TRAJ" gpurun_out/r6v_pytest.log | cut -c1-300
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6v_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r6v_smoke.log; exit 1; }
tail -1 gpurun_out/r6v_smoke.log | cut -c1-200
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6v_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r6v_bench.log; exit 1; }
grep '^{' gpurun_out/r6v_bench.log | cut -c1-400
