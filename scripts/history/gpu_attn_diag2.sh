# dQ-kernel skeleton split: everything skipped but the prologue (Q / dO / O loads, delta) and the epilogue
set -o pipefail
mkdir -p gpurun_out
for d in 39 36 0; do
  DALLE_AMD_ATTN_DIAG=$d timeout -k 10 120 python3 -u benchmarks/bench_attn_parts.py 128 > gpurun_out/attn_diag2_$d.log 2>&1 || { echo "diag $d failed"; tail -5 gpurun_out/attn_diag2_$d.log; exit 1; }
  echo "diag=$d"; grep '^{' gpurun_out/attn_diag2_$d.log
done
