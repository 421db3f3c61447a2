set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY TCC_HIT_sum TCC_MISS_sum --stats -d gpurun_out/pmc_a -o run --output-format csv -- python3 benchmarks/bench_ops.py --only attn > gpurun_out/pmc_a.log 2>&1 || { echo "pmc a failed"; tail -20 gpurun_out/pmc_a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --stats -d gpurun_out/pmc_b -o run --output-format csv -- python3 benchmarks/bench_ops.py --only attn > gpurun_out/pmc_b.log 2>&1 || { echo "pmc b failed"; tail -20 gpurun_out/pmc_b.log; exit 1; }
echo done
