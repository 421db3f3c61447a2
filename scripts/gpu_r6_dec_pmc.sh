# round 6: PMC passes over the decode kernels (reference model, batch 64, repeated caption, 8 eager image-position steps:
# counter collection under hipGraph replay crashed the profiler)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
pass() {  # name, counters
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$name -o run --output-format csv -- python3 benchmarks/bench_inference.py --batch 64 --profile-steps 8 --no-vae --same-caption --no-graph > gpurun_out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 gpurun_out/pmc_$name.log; exit 1; }
}
pass d1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM
pass d2 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACCUM_PREV_HIRES SQ_LEVEL_WAVES
python3 scripts/pmc_raw.py gpurun_out/pmc_d1 gpurun_out/pmc_d2 > gpurun_out/r6_dec_pmc.txt 2>&1 || true
grep -A 18 "decode_attn\|skinny_gemm_kernel<2, 1, 4, 2>\|decode_ln" gpurun_out/r6_dec_pmc.txt | head -80
