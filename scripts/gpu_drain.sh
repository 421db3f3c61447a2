# GEMM end-of-workgroup store drain A/B + GEMM tests + full-step benches under GEMM routing options
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_pt_gpu.py tests/test_fused_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/drain_test.log 2>&1 || { echo "gemm tests failed"; tail -40 gpurun_out/drain_test.log; exit 1; }
tail -1 gpurun_out/drain_test.log
timeout -k 10 500 python3 -u benchmarks/bench_gemm_drain.py > gpurun_out/drain_bench.log 2>&1 || { echo "drain bench failed"; tail -30 gpurun_out/drain_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/drain_bench.log
for cfg in "DALLE_AMD_GEMM_DRAIN=1" "DALLE_AMD_GEMM_DRAIN=0" "DALLE_AMD_OWN_GEMM=1" "DALLE_AMD_OWN_GEMM=1 DALLE_AMD_FUSED_FF_IN=1" "DALLE_AMD_OWN_GEMM=1 DALLE_AMD_FUSED_FF_IN=1 DALLE_AMD_OWN_WGRAD=1"; do
  env $cfg timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > gpurun_out/drain_step.log 2>&1 || { echo "bench failed ($cfg)"; tail -20 gpurun_out/drain_step.log; exit 1; }
  echo "$cfg $(grep '^{' gpurun_out/drain_step.log | cut -c120-200)"
done
