# Attention time split by part (measurement only): bench_attn_parts at B128 with DALLE_AMD_ATTN_DIAG
# skipping pieces -- 1 text staging, 2 its barriers, 4 local tiles, 32 text compute (fwd / dQ);
# 8 staging, 16 barriers (text dK/dV). Results are NOT numerically meaningful with diag != 0.
set -o pipefail
mkdir -p gpurun_out
for d in 0 1 2 3 4 32 36 24; do
  DALLE_AMD_ATTN_DIAG=$d timeout -k 10 120 python3 -u benchmarks/bench_attn_parts.py 128 > gpurun_out/attn_diag_$d.log 2>&1 || { echo "diag $d failed"; tail -5 gpurun_out/attn_diag_$d.log; exit 1; }
  echo "diag=$d"; grep '^{' gpurun_out/attn_diag_$d.log
done
