# register-epilogue GEGLU-backward GEMM (one tile per workgroup) under different tile orders (DALLE_AMD_PT_GROUP)
set -o pipefail
mkdir -p gpurun_out
for v in 4 1 2 8 16 -1 -4 -16; do
  DALLE_AMD_PT_GROUP=$v timeout -k 10 200 python3 -u benchmarks/bench_geglu_bwd_variants.py > gpurun_out/geglu_group.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/geglu_group.log; exit 1; }
  echo "group=$v $(grep '^{"M"' gpurun_out/geglu_group.log)"
done
