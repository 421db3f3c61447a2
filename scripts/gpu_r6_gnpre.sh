# round 6: VQGAN GroupNorm + SiLU as a pre-pass (gn_apply silu) ahead of the plain 3x3 conv vs fused into the gather,
# by image-size threshold; decoder tests with the pre-pass everywhere
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
DALLE_AMD_VQGAN_GN_PREPASS=0 timeout -k 10 400 python3 -u -m pytest tests/test_vqgan_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6gn_pytest.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/r6gn_pytest.log; exit 1; }
tail -1 gpurun_out/r6gn_pytest.log
for rep in 1 2; do
  for thr in never 65536 16384 4096 0; do
    if [ "$thr" = never ]; then unset DALLE_AMD_VQGAN_GN_PREPASS; else export DALLE_AMD_VQGAN_GN_PREPASS=$thr; fi
    timeout -k 10 200 python3 benchmarks/bench_vqgan.py --iters 5 > gpurun_out/r6gn_vq.log 2>&1 || { echo "vq $thr failed"; tail -5 gpurun_out/r6gn_vq.log; exit 1; }
    echo "thr=$thr $(grep '^{' gpurun_out/r6gn_vq.log | grep -oE '"hip_ms": [0-9.]+')"
  done
done
