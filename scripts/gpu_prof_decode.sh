set -o pipefail
# kernel trace of eager decode steps at image positions (prefill + 48 steps), batch 64 and 32
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 64 32; do
  DALLE_AMD_DECODE_PARTS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dec$b -o run --output-format csv -- python3 benchmarks/bench_inference.py --batch $b --model reference --profile-steps 48 --no-vae > gpurun_out/prof_dec$b.log 2>&1 || { echo "prof $b failed"; tail -20 gpurun_out/prof_dec$b.log; exit 1; }
  rm -f gpurun_out/prof_dec$b/run_kernel_trace.csv
  python3 scripts/prof_summary.py gpurun_out/prof_dec$b/run_kernel_stats.csv 12 1 > gpurun_out/prof_dec${b}_top.txt
  head -14 gpurun_out/prof_dec${b}_top.txt | cut -c1-150
done
