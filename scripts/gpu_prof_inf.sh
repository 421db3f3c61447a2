set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_inf -o run --output-format csv -- python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 --no-vae > gpurun_out/prof_inf.log 2>&1 || { echo "prof inf failed"; tail -20 gpurun_out/prof_inf.log; exit 1; }
rm -f gpurun_out/prof_inf/run_kernel_trace.csv
grep "#\|{" gpurun_out/prof_inf.log | cut -c1-300
