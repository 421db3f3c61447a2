# kernel trace of the bench step (5 timed steps) -> profiles summary
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
rm -f gpurun_out/prof_$TAG/run_kernel_trace.csv
grep metric gpurun_out/prof_$TAG.log | cut -c1-300
python3 scripts/prof_summary.py gpurun_out/prof_$TAG/run_kernel_stats.csv 40 7 > gpurun_out/prof_${TAG}_top.txt
head -45 gpurun_out/prof_${TAG}_top.txt
