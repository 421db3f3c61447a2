# kernel profile of the ~1.3B reversible config (BASELINE config 4) at micro-batch 32
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --model dalle-1.3b --batch 32 --steps 6 --warmup 2 > gpurun_out/b13.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/b13.log; exit 1; }
grep '^{' gpurun_out/b13.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_b13 -o run --output-format csv -- python3 bench.py --model dalle-1.3b --batch 32 --steps 3 --warmup 2 > gpurun_out/prof_b13.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_b13.log; exit 1; }
rm -f gpurun_out/prof_b13/run_kernel_trace.csv
python3 scripts/prof_summary.py gpurun_out/prof_b13/run_kernel_stats.csv 30 5 > gpurun_out/prof_b13_top.txt
head -31 gpurun_out/prof_b13_top.txt | cut -c1-160
