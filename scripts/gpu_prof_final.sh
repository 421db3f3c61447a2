set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_final.log 2>&1 || { echo "rocprof train failed"; tail -20 gpurun_out/prof_final.log; exit 1; }
rm -f gpurun_out/prof_final/run_kernel_trace.csv
grep metric gpurun_out/prof_final.log | cut -c1-200
python3 scripts/prof_summary.py gpurun_out/prof_final/run_kernel_stats.csv 30 7
