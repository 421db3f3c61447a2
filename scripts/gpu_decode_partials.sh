set -o pipefail
# decode with split-K partials: GPU generation tests, then reference-model inference A/B (same box)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_generation_gpu.py tests/test_skinny_gpu.py > gpurun_out/part_tests.log 2>&1 || { tail -40 gpurun_out/part_tests.log; exit 1; }
tail -1 gpurun_out/part_tests.log
for v in 0 1; do
  DALLE_AMD_DECODE_PARTIALS=$v timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 > gpurun_out/inf_part$v.log 2>&1 || { echo "inference $v failed"; tail -20 gpurun_out/inf_part$v.log; exit 1; }
  echo "partials=$v $(grep metric gpurun_out/inf_part$v.log | cut -c1-260)"
done
