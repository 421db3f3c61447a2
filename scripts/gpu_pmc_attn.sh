set -o pipefail
# attention kernels: per-op times at B48 + MFMA / VALU / LDS counters (one counter pass per run)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python3 benchmarks/bench_ops.py --only attn --batch 48 > gpurun_out/ops_attn.log 2>&1 || { echo "bench_ops failed"; tail -20 gpurun_out/ops_attn.log; exit 1; }
cat gpurun_out/ops_attn.log | grep -v amdgpu.ids
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace -d gpurun_out/pmc_a -o run --output-format csv -- python3 benchmarks/bench_ops.py --only attn --batch 48 > gpurun_out/pmc_a.log 2>&1 || { echo "pmc a failed"; tail -20 gpurun_out/pmc_a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmc_b -o run --output-format csv -- python3 benchmarks/bench_ops.py --only attn --batch 48 > gpurun_out/pmc_b.log 2>&1 || { echo "pmc b failed"; tail -20 gpurun_out/pmc_b.log; exit 1; }
echo done
