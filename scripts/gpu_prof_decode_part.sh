set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
  DALLE_AMD_DECODE_PARTIALS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dp$v -o run --output-format csv -- python3 benchmarks/bench_inference.py --batch 64 --model reference --profile-steps 48 --no-vae > gpurun_out/prof_dp$v.log 2>&1 || { echo "prof $v failed"; tail -20 gpurun_out/prof_dp$v.log; exit 1; }
  rm -f gpurun_out/prof_dp$v/run_kernel_trace.csv
  python3 scripts/prof_summary.py gpurun_out/prof_dp$v/run_kernel_stats.csv 10 1 > gpurun_out/prof_dp${v}_top.txt
  head -11 gpurun_out/prof_dp${v}_top.txt | cut -c1-140
done
