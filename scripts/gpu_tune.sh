set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --tunable off > gpurun_out/bench_off.log 2>&1 || { echo "bench off failed"; tail -20 gpurun_out/bench_off.log; exit 1; }
tail -1 gpurun_out/bench_off.log
timeout -k 10 900 python3 bench.py --steps 2 --warmup 2 --tunable tune > gpurun_out/bench_tune.log 2>&1 || { echo "bench tune failed"; tail -20 gpurun_out/bench_tune.log; exit 1; }
ls -la profiles/tunableop_gfx950.csv && cp profiles/tunableop_gfx950.csv gpurun_out/
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --tunable use > gpurun_out/bench_use.log 2>&1 || { echo "bench use failed"; tail -20 gpurun_out/bench_use.log; exit 1; }
tail -1 gpurun_out/bench_use.log
