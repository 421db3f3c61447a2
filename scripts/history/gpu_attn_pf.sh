# attention: local-tile prefetch before the text phase, by occupancy (bench_attn_parts at micro-batch 128)
set -o pipefail
mkdir -p gpurun_out
for cfg in "3,3,2,2 0,0" "3,3,2,2 1,0" "2,3,2,2 1,0" "3,3,2,2 0,1" "3,2,2,2 0,1" "3,2,2,2 0,0"; do
  set -- $cfg
  DALLE_AMD_ATTN_OCC=$1 DALLE_AMD_ATTN_PF=$2 timeout -k 10 120 python3 benchmarks/bench_attn_parts.py 128 > gpurun_out/attn_pf_${1}_${2}.log 2>&1 || { echo "failed $cfg"; tail -5 gpurun_out/attn_pf_${1}_${2}.log; exit 1; }
  echo "occ=$1 pf=$2: $(grep -h '^{' gpurun_out/attn_pf_${1}_${2}.log | tr '\n' ' ' | cut -c1-600)"
done
