# decode at image positions: inference bench (reference model, batch 64) + kernel profile of 64 image steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 > gpurun_out/inf_img.log 2>&1 || { echo "inference failed"; tail -20 gpurun_out/inf_img.log; exit 1; }
grep -h '^#\|metric' gpurun_out/inf_img.log | cut -c1-330
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_img -o run --output-format csv -- python3 benchmarks/bench_inference.py --batch 64 --model reference --profile-steps 64 --no-vae > gpurun_out/prof_img.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_img.log; exit 1; }
rm -f gpurun_out/prof_img/run_kernel_trace.csv
python3 scripts/prof_summary.py gpurun_out/prof_img/run_kernel_stats.csv 16 1 > gpurun_out/prof_img_top.txt
head -17 gpurun_out/prof_img_top.txt | cut -c1-150
