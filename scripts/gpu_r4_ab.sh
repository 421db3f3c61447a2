# Round-4 A/B on one box: smoke, the register-epilogue GEGLU tests, the GEGLU variants benchmark, the
# attention start-stagger test, then the bench step at the defaults and under the candidate switches.
# usage: bash scripts/gpu_r4_ab.sh TAG
set -o pipefail
TAG=${1:-r4ab}
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log | cut -c1-200
{ timeout -k 10 300 python3 -u -m pytest tests/test_gemm_pt_gpu.py -x -q --timeout 120 --timeout-method thread -k "dgrad or line_stores or ff_in" && timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "four_tiles or three_tiles or dma_staging or sparse_attention"; } > gpurun_out/${TAG}_pt_tests.log 2>&1 || { echo "pt tests failed"; tail -30 gpurun_out/${TAG}_pt_tests.log; exit 1; }
grep -E 'passed|failed' gpurun_out/${TAG}_pt_tests.log
timeout -k 10 300 python3 -u benchmarks/bench_geglu_bwd_variants.py > gpurun_out/${TAG}_geglu_variants.jsonl 2>&1 || { echo "geglu bench failed"; tail -5 gpurun_out/${TAG}_geglu_variants.jsonl; exit 1; }
cat gpurun_out/${TAG}_geglu_variants.jsonl
step() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench_$name.log 2>&1 || { echo "bench $name failed"; tail -20 gpurun_out/${TAG}_bench_$name.log; exit 1; }
  echo "$name $(grep '^{' gpurun_out/${TAG}_bench_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
step default X=1
step geglu_pt DALLE_AMD_GEGLU_DGRAD_KERNEL=pt
step ffin_pt DALLE_AMD_FUSED_FF_IN=1
step dkdv_qt4 DALLE_AMD_DKDV_QT=4
step fwd_tps3 DALLE_AMD_ATTN_FWD_TPS=3
step dq_stage3 DALLE_AMD_ATTN_DQ_STAGE=3
step default2 X=1
bash scripts/gpu_attn_stagger.sh
