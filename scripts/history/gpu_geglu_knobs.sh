# GEGLU-backward GEMM (8-phase vs register-epilogue one tile per workgroup) under the store knobs
set -o pipefail
mkdir -p gpurun_out
for v in "X=0" "DALLE_AMD_GEMM_DRAIN=0" "DALLE_AMD_GEMM_CPOL=2" "DALLE_AMD_GEMM_CPOL=17" "DALLE_AMD_GEMM_DRAIN=0 DALLE_AMD_GEMM_CPOL=2"; do
  env $v timeout -k 10 200 python3 -u benchmarks/bench_geglu_bwd_variants.py > gpurun_out/geglu_knob.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/geglu_knob.log; exit 1; }
  echo "$v $(grep '^{"M"' gpurun_out/geglu_knob.log)"
done
