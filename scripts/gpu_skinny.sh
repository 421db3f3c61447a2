set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_skinny_gpu.py tests/test_generation_gpu.py -x -q > gpurun_out/skinny_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/skinny_tests.log; exit 1; }
tail -2 gpurun_out/skinny_tests.log
timeout -k 10 300 python benchmarks/bench_skinny.py --batch 64 > gpurun_out/bench_skinny.log 2>&1 || { echo "bench_skinny failed"; tail -20 gpurun_out/bench_skinny.log; exit 1; }
grep "{" gpurun_out/bench_skinny.log
timeout -k 10 600 python benchmarks/bench_inference.py --batch 64 --model reference --iters 1 --no-vae > gpurun_out/inf_skinny.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/inf_skinny.log; exit 1; }
grep "#\|{" gpurun_out/inf_skinny.log | cut -c1-300
timeout -k 10 600 python benchmarks/bench_inference.py --batch 64 --model bench24 --iters 1 --no-vae > gpurun_out/inf_skinny24.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/inf_skinny24.log; exit 1; }
grep "{" gpurun_out/inf_skinny24.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_inf -o run --output-format csv -- python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 --no-vae > gpurun_out/prof_inf.log 2>&1 || { echo "prof inf failed"; tail -20 gpurun_out/prof_inf.log; exit 1; }
rm -f gpurun_out/prof_inf/run_kernel_trace.csv
