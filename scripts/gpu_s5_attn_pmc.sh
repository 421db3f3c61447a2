set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "attention or rotary" > gpurun_out/pytest_attn3.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_attn3.log; exit 1; }
tail -1 gpurun_out/pytest_attn3.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc_attn5 -o run --output-format csv -- python3 benchmarks/bench_ops.py --only attn --batch 48 > gpurun_out/pmc_attn5.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_attn5.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/pmc_attn5 --top 8
