set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/prof_train.log 2>&1 || { echo "rocprof train failed"; tail -20 gpurun_out/prof_train.log; exit 1; }
tail -1 gpurun_out/prof_train.log
