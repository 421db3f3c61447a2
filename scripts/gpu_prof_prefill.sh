# batched caption prefill: wall time + kernel profile (reference model, batch 64)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 benchmarks/bench_prefill.py > gpurun_out/prefill.log 2>&1 || { tail -20 gpurun_out/prefill.log; exit 1; }
grep prefill_ms gpurun_out/prefill.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pf -o run --output-format csv -- python3 benchmarks/bench_prefill.py > gpurun_out/prof_pf.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_pf.log; exit 1; }
rm -f gpurun_out/prof_pf/run_kernel_trace.csv
python3 scripts/prof_summary.py gpurun_out/prof_pf/run_kernel_stats.csv 16 5 > gpurun_out/prof_pf_top.txt
head -18 gpurun_out/prof_pf_top.txt | cut -c1-150
