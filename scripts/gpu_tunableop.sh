set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTORCH_TUNABLEOP_VERBOSE=1
( while sleep 50; do echo "heartbeat $(date +%T)"; done ) &
HB=$!
trap 'kill $HB' EXIT
timeout -k 10 900 python3 bench.py --tunable tune --steps 2 --warmup 1 > gpurun_out/tune.log 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tune.log; exit 1; }
cp profiles/tunableop_gfx950.csv gpurun_out/ || exit 1
grep '^{' gpurun_out/tune.log | cut -c1-160
unset PYTORCH_TUNABLEOP_VERBOSE
timeout -k 10 300 python3 bench.py --tunable use --steps 10 --warmup 3 > gpurun_out/tuned.log 2>&1 || { echo "tuned bench failed"; tail -20 gpurun_out/tuned.log; exit 1; }
grep '^{' gpurun_out/tuned.log | cut -c1-220
timeout -k 10 300 python3 bench.py --tunable off --steps 10 --warmup 3 > gpurun_out/untuned.log 2>&1 || { echo "untuned bench failed"; tail -20 gpurun_out/untuned.log; exit 1; }
grep '^{' gpurun_out/untuned.log | cut -c1-220
