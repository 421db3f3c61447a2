set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -m pytest tests/test_kernels_gpu.py tests/test_fused_gpu.py tests/test_model_gpu.py -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python3 benchmarks/bench_ops.py --only attn > gpurun_out/attn.log 2>&1 || { echo "attn bench failed"; tail -20 gpurun_out/attn.log; exit 1; }
grep op gpurun_out/attn.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/bench16.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench16.log; exit 1; }
tail -1 gpurun_out/bench16.log
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --stats -d gpurun_out/pmc_attn -o run --output-format csv -- python3 benchmarks/bench_ops.py --only attn > gpurun_out/pmc_attn.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_attn.log; exit 1; }
