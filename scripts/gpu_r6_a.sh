# round 6, first GPU pass: full GPU suite (per-class gradient errors logged), bench24, the ~1.3B config on the
# assembly kernels (K = 2048) and its kernel table
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r6a_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/r6a_pytest.log | head -30; tail -30 gpurun_out/r6a_pytest.log; exit 1; }
tail -2 gpurun_out/r6a_pytest.log
grep GRAD_ERR gpurun_out/r6a_pytest.log | cut -c1-600
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6a_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r6a_bench.log; exit 1; }
grep '^{' gpurun_out/r6a_bench.log | cut -c1-300
timeout -k 10 400 python3 bench.py --model dalle-1.3b --batch 32 --steps 3 --warmup 1 --recompute auto > gpurun_out/r6a_l13.log 2>&1 || { echo "l13 failed"; tail -20 gpurun_out/r6a_l13.log; exit 1; }
grep '^{' gpurun_out/r6a_l13.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6_l13 -o run --output-format csv -- python3 bench.py --model dalle-1.3b --batch 32 --steps 3 --warmup 2 --recompute auto > gpurun_out/prof_r6_l13.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_r6_l13.log; exit 1; }
rm -f gpurun_out/prof_r6_l13/run_kernel_trace.csv
python3 scripts/prof_summary.py gpurun_out/prof_r6_l13/run_kernel_stats.csv 30 5 > gpurun_out/prof_r6_l13_top.txt
head -31 gpurun_out/prof_r6_l13_top.txt | cut -c1-160
