# round 6: step kernel tables with the fused attention backward on / off, and LN-shift byte counters
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in 1 0; do
  DALLE_AMD_ATTN_FUSED_BWD=$f timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6_step_f$f -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > gpurun_out/prof_r6_step_f$f.log 2>&1 || { echo "prof $f failed"; tail -20 gpurun_out/prof_r6_step_f$f.log; exit 1; }
  rm -f gpurun_out/prof_r6_step_f$f/run_kernel_trace.csv
  python3 scripts/prof_summary.py gpurun_out/prof_r6_step_f$f/run_kernel_stats.csv 16 5 > gpurun_out/prof_r6_step_f${f}_top.txt
  echo "fused=$f"; head -17 gpurun_out/prof_r6_step_f${f}_top.txt | cut -c1-150
done
for c in FETCH_SIZE WRITE_SIZE; do timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/pmc_ln_$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 > gpurun_out/pmc_ln_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 gpurun_out/pmc_ln_$c.log; exit 1; }; done
python3 scripts/pmc_raw.py gpurun_out/pmc_ln_FETCH_SIZE gpurun_out/pmc_ln_WRITE_SIZE | grep -A 2 "ln_shift" | head -24
