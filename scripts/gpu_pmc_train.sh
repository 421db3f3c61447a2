set -o pipefail
# hardware counters of one bench24 training run per counter group (one --pmc pass each)
mkdir -p gpurun_out
export TMPDIR=/tmp
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-trace -d gpurun_out/pmc_r2s4_$name -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > gpurun_out/pmc_r2s4_$name.log 2>&1 || { echo "pmc $name failed"; tail -20 gpurun_out/pmc_r2s4_$name.log; exit 1; }
  rm -f gpurun_out/pmc_r2s4_$name/run_kernel_trace.csv
}
pass mfma SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 scripts/pmc_summary.py gpurun_out/pmc_r2s4_mfma gpurun_out/pmc_r2s4_fetch gpurun_out/pmc_r2s4_write --top 24
