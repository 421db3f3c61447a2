set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 benchmarks/bench_ops.py --only attn > gpurun_out/attn.log 2>&1 || { echo "attn bench failed"; tail -20 gpurun_out/attn.log; exit 1; }
grep op gpurun_out/attn.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_attn -o run --output-format csv -- python3 benchmarks/bench_ops.py --only attn > gpurun_out/prof_attn.log 2>&1 || { echo "prof failed"; exit 1; }
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/bench16.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench16.log; exit 1; }
tail -1 gpurun_out/bench16.log
