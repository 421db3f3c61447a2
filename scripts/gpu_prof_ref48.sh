# kernel profile of the reference recipe (64 layers, 5 shared blocks, reversible, auto activation store) at micro-batch 48
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --model reference --batch 48 --recompute auto --steps 6 --warmup 2 > gpurun_out/ref48.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/ref48.log; exit 1; }
grep '^{' gpurun_out/ref48.log | cut -c1-400
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ref48 -o run --output-format csv -- python3 bench.py --model reference --batch 48 --recompute auto --steps 3 --warmup 2 > gpurun_out/prof_ref48.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_ref48.log; exit 1; }
rm -f gpurun_out/prof_ref48/run_kernel_trace.csv
python3 scripts/prof_summary.py gpurun_out/prof_ref48/run_kernel_stats.csv 30 5 > gpurun_out/prof_ref48_top.txt
head -31 gpurun_out/prof_ref48_top.txt | cut -c1-160
