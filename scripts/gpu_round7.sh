set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/bench16.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench16.log; exit 1; }
tail -1 gpurun_out/bench16.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof_train.log 2>&1 || { echo "rocprof train failed"; tail -20 gpurun_out/prof_train.log; exit 1; }
BENCH_BATCH=32 timeout -k 10 300 python3 bench.py --steps 8 --warmup 3 > gpurun_out/bench32.log 2>&1 || { echo "bench32 failed"; tail -20 gpurun_out/bench32.log; exit 1; }
tail -1 gpurun_out/bench32.log
