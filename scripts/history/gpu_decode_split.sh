set -o pipefail
# split decode engine: GPU tests, then reference-model inference at batch 64 with 1 and 2 parts
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_generation_gpu.py > gpurun_out/split_tests.log 2>&1 || { tail -40 gpurun_out/split_tests.log; exit 1; }
tail -2 gpurun_out/split_tests.log
for parts in 1 2 4; do
  DALLE_AMD_DECODE_PARTS=$parts timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 > gpurun_out/inf_parts$parts.log 2>&1 || { echo "parts $parts failed"; tail -20 gpurun_out/inf_parts$parts.log; exit 1; }
  grep metric gpurun_out/inf_parts$parts.log | cut -c1-420
done
