set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_skinny_gpu.py -x -q > gpurun_out/skinny_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/skinny_tests.log; exit 1; }
tail -2 gpurun_out/skinny_tests.log
timeout -k 10 600 python benchmarks/bench_skinny.py --batch 64 --ablate > gpurun_out/bench_skinny_sweep.log 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/bench_skinny_sweep.log; exit 1; }
grep "{" gpurun_out/bench_skinny_sweep.log
