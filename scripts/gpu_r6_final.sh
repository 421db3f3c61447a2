# round 6 final-tree check: full GPU suite (pinned per-class gradient bounds, 20-step LAMB trajectory), smoke, bench24
# (driver form), the 1.3B config, and the LN-shift byte counters
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r6f_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r6f_pytest.log | head -30; tail -30 gpurun_out/r6f_pytest.log; exit 1; }
tail -2 gpurun_out/r6f_pytest.log
grep -E "GRAD_ERR|TRAJ" gpurun_out/r6f_pytest.log | cut -c1-300
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6f_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r6f_smoke.log; exit 1; }
tail -1 gpurun_out/r6f_smoke.log | cut -c1-200
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6f_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r6f_bench.log; exit 1; }
grep '^{' gpurun_out/r6f_bench.log | cut -c1-400
timeout -k 10 400 python3 bench.py --model dalle-1.3b --batch 32 --steps 3 --warmup 1 --recompute auto > gpurun_out/r6f_l13.log 2>&1 || { echo "l13 failed"; tail -20 gpurun_out/r6f_l13.log; exit 1; }
grep '^{' gpurun_out/r6f_l13.log | cut -c1-300
for c in FETCH_SIZE WRITE_SIZE; do timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmc_ln_$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pmc_ln_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_ln_$c.log; exit 1; }; done
python3 scripts/pmc_raw.py gpurun_out/pmc_ln_FETCH_SIZE gpurun_out/pmc_ln_WRITE_SIZE > gpurun_out/r6f_pmc_bytes.txt
grep -A 2 "ln_shift" gpurun_out/r6f_pmc_bytes.txt | head -24
