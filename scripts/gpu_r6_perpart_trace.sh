# round 6: kernel trace of the per-part decode graphs (two half-batch chains, each a linear graph on its own stream),
# repeated caption, last 24 of 48 image-position steps
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_pp -o run --output-format csv -- python3 $R/benchmarks/bench_inference.py --batch 64 --model reference --profile-steps 48 --no-vae --same-caption > $R/gpurun_out/prof_pp.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_pp.log; exit 1; }
cd $R
python3 scripts/decode_trace_summary.py gpurun_out/prof_pp/run_kernel_trace.csv --steps 24 --chains 2 > gpurun_out/r6pp_trace_summary.txt
rm -f gpurun_out/prof_pp/run_kernel_trace.csv
head -30 gpurun_out/r6pp_trace_summary.txt
