# attention occupancy variants (DALLE_AMD_ATTN_OCC=fwd,dq,dkdv_text,dkdv) on the final round-4 kernels, parts bench B128, twice each
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for o in 3,3,2,2 2,3,2,2 3,2,2,2 2,2,2,2 3,3,2,2 2,3,2,2 3,2,2,2 2,2,2,2; do
  DALLE_AMD_ATTN_OCC=$o timeout -k 10 120 python3 -u benchmarks/bench_attn_parts.py 128 > gpurun_out/occ_$o.log 2>&1 || { echo "occ $o failed"; tail -5 gpurun_out/occ_$o.log; exit 1; }
  echo "occ=$o $(grep -h 'bench24_attention' gpurun_out/occ_$o.log) $(grep -h axial_row gpurun_out/occ_$o.log)"
done
