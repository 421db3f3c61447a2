# Attention lockstep test (measurement): bench_attn_parts at B128 with the first-round start stagger
set -o pipefail
mkdir -p gpurun_out
for t in 0 300 600 1000; do
  DALLE_AMD_ATTN_STAGGER=$t timeout -k 10 120 python3 -u benchmarks/bench_attn_parts.py 128 > gpurun_out/attn_stagger_$t.log 2>&1 || { echo "stagger $t failed"; tail -5 gpurun_out/attn_stagger_$t.log; exit 1; }
  echo "stagger=$t"; grep '^{' gpurun_out/attn_stagger_$t.log
done
for v in "DALLE_AMD_ATTN_FWD_TPS=3" "DALLE_AMD_DKDV_QT=4" "DALLE_AMD_ATTN_DQ_STAGE=2" "DALLE_AMD_ATTN_DQ_STAGE=3" "X=0"; do
  env $v timeout -k 10 120 python3 -u benchmarks/bench_attn_parts.py 128 > gpurun_out/attn_var_${v//=/_}.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/attn_var_${v//=/_}.log; exit 1; }
  echo "$v"; grep '^{' gpurun_out/attn_var_${v//=/_}.log
done
