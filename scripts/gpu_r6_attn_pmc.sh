# round 6: PMC passes over the fused attention backward (and the two-kernel form) at B128, axial_row
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
pass() {  # name, env, counters
  local name=$1 envv=$2; shift 2
  env $envv timeout -s KILL 90 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$name -o run --output-format csv -- python3 benchmarks/attn_bwd_once.py axial_row 3 128 > gpurun_out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/pmc_$name.log; exit 1; }
}
pass f1 DALLE_AMD_ATTN_FUSED_BWD=1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA
pass f2 DALLE_AMD_ATTN_FUSED_BWD=1 SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU
pass f3 DALLE_AMD_ATTN_FUSED_BWD=1 FETCH_SIZE TCC_EA0_WRREQ_sum
pass t1 DALLE_AMD_ATTN_FUSED_BWD=0 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA
python3 scripts/pmc_raw.py gpurun_out/pmc_f1 gpurun_out/pmc_f2 gpurun_out/pmc_f3 gpurun_out/pmc_t1 > gpurun_out/r6_attn_pmc.txt 2>&1 || true
cat gpurun_out/r6_attn_pmc.txt | head -60
