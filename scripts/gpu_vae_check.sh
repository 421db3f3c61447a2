# VQGAN decoder standalone + where generate_images' non-sampling time goes (rocprof of one generate)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 benchmarks/bench_vqgan.py > gpurun_out/vae.log 2>&1 || { echo "vae bench failed"; tail -20 gpurun_out/vae.log; exit 1; }
grep '^{' gpurun_out/vae.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_inf -o run --output-format csv -- python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 > gpurun_out/prof_inf.log 2>&1 || { echo "rocprof inf failed"; tail -20 gpurun_out/prof_inf.log; exit 1; }
rm -f gpurun_out/prof_inf/run_kernel_trace.csv
grep metric gpurun_out/prof_inf.log | cut -c1-200
python3 scripts/prof_summary.py gpurun_out/prof_inf/run_kernel_stats.csv 30 1 > gpurun_out/prof_inf_top.txt; head -32 gpurun_out/prof_inf_top.txt
