set -o pipefail
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
DALLE_AMD_BACKEND=torch timeout -k 10 600 python bench.py --steps 4 --warmup 2 --batch 8 > gpurun_out/bench_torch.log 2>&1
echo EXIT $?
tail -5 gpurun_out/bench_torch.log
