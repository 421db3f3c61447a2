set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests/test_kernels_gpu.py -x -q -k "attention" > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 benchmarks/bench_ops.py --only attn > gpurun_out/attn.log 2>&1 || { echo "attn bench failed"; tail -20 gpurun_out/attn.log; exit 1; }
grep op gpurun_out/attn.log
