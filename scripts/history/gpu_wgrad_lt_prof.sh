# kernel tables of the bench step with / without the measured-solution weight grads
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0; do
  DALLE_AMD_WGRAD_LT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wlt$v -o run --output-format csv -- python3 bench.py --steps 4 --warmup 2 > gpurun_out/prof_wlt$v.log 2>&1 || { echo "prof $v failed"; tail -20 gpurun_out/prof_wlt$v.log; exit 1; }
  rm -f gpurun_out/prof_wlt$v/run_kernel_trace.csv
  python3 scripts/prof_summary.py gpurun_out/prof_wlt$v/run_kernel_stats.csv 30 6 > gpurun_out/prof_wlt${v}_top.txt
  echo "== lt=$v"; grep -E "Cijk|splitk|all kernels" gpurun_out/prof_wlt${v}_top.txt | cut -c1-160
done
