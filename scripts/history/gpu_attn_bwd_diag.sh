# attention backward per-kernel times with measurement-only phase skips (DALLE_AMD_ATTN_DIAG)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in ${DIAGS:-0 1 3 4 8 24}; do
  DALLE_AMD_ATTN_DIAG=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/bwddiag_$d -o run --output-format csv -- python3 benchmarks/attn_bwd_diag.py > gpurun_out/bwddiag_$d.log 2>&1 || { echo "diag $d failed"; tail -20 gpurun_out/bwddiag_$d.log; exit 1; }
  f=$(find gpurun_out/bwddiag_$d -name '*kernel_stats.csv' | head -1)
  echo "== diag $d"; grep -E "attn_bwd|attn_delta" "$f" | cut -d, -f1-5
done
