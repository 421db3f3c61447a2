set -o pipefail
# one counter pass over the weight-grad kernels (hand-written MN-major vs hipBLASLt vs NT), then the sweep
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_gpu.py -k "wgrad" > gpurun_out/wgrad_tests.log 2>&1 || { tail -30 gpurun_out/wgrad_tests.log; exit 1; }
tail -2 gpurun_out/wgrad_tests.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_wgrad -o run --output-format csv -- python3 benchmarks/bench_wgrad_kernel.py 61440 1024 4096 4 > gpurun_out/pmc_wgrad.log 2>&1 || { echo "pmc failed"; tail -20 gpurun_out/pmc_wgrad.log; exit 1; }
rm -f gpurun_out/pmc_wgrad/run_kernel_trace.csv
python3 scripts/pmc_summary.py gpurun_out/pmc_wgrad --top 8
timeout -k 10 300 python benchmarks/bench_gemm.py --wgrad > gpurun_out/wgrad_bench.jsonl 2>&1 && cat gpurun_out/wgrad_bench.jsonl
