set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_sampler_gpu.py tests/test_generation_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sampler.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_sampler.log; exit 1; }
tail -4 gpurun_out/pytest_sampler.log
timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 2 > gpurun_out/inf_ref_fused.log 2>&1 || { echo "bench inf failed"; tail -20 gpurun_out/inf_ref_fused.log; exit 1; }
grep -v amdgpu.ids gpurun_out/inf_ref_fused.log | tail -5
DALLE_AMD_FUSED_SAMPLER=0 timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 2 > gpurun_out/inf_ref_torchsampler.log 2>&1 || { echo "bench inf (torch sampler) failed"; tail -20 gpurun_out/inf_ref_torchsampler.log; exit 1; }
grep -v amdgpu.ids gpurun_out/inf_ref_torchsampler.log | tail -5
