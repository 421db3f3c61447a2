# dQ-kernel skeleton split further (measurement only): 39 = no text staging / barriers / local / text compute;
# +64 no fused local dK/dV; +128 no dQ stores
set -o pipefail
mkdir -p gpurun_out
for d in 39 103 167 231; do
  DALLE_AMD_ATTN_DIAG=$d timeout -k 10 120 python3 -u benchmarks/bench_attn_parts.py 128 > gpurun_out/attn_diag3_$d.log 2>&1 || { echo "diag $d failed"; tail -5 gpurun_out/attn_diag3_$d.log; exit 1; }
  echo "diag=$d"; grep '^{"pattern": "axial_row"' gpurun_out/attn_diag3_$d.log
done
