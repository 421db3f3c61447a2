# attention forward / dQ with the compute skipped (prologue + epilogue cost) and other phase skips
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 7 39 35; do
  DALLE_AMD_ATTN_DIAG=$d timeout -k 10 120 python3 benchmarks/attn_fwd_diag.py || exit 1
done
DIAGS="7 39" bash scripts/gpu_attn_bwd_diag.sh
