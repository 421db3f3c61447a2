# dQ kernel VALU / MFMA instruction counts per part (PMC), bench_attn_parts B128 axial patterns:
# diag 0 = all, 64 = no fused local dK/dV, 4 = no local tiles, 32 = no text-tile compute, 128 = no dQ stores
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in 0 64 4 32 128; do
  DALLE_AMD_ATTN_DIAG=$d timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/dqvalu_$d -o run --output-format csv -- python3 benchmarks/bench_attn_parts.py 128 > gpurun_out/dqvalu_$d.log 2>&1 || { echo "pmc $d failed"; tail -5 gpurun_out/dqvalu_$d.log; exit 1; }
  rm -f gpurun_out/dqvalu_$d/*/run_kernel_trace.csv gpurun_out/dqvalu_$d/run_kernel_trace.csv
  echo "diag $d done"
done
