# decode kernel trace (reference model, batch 64, 32 image-position steps): per-kernel durations and the timeline
set -o pipefail
mkdir -p gpurun_out
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_dec -o run --output-format csv -- python3 $R/benchmarks/bench_inference.py --batch 64 --model reference --profile-steps 32 --no-vae > $R/gpurun_out/prof_dec.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_dec.log; exit 1; }
cd $R && ls -la gpurun_out/prof_dec
python3 scripts/decode_trace_summary.py gpurun_out/prof_dec/run_kernel_trace.csv --steps 16 > gpurun_out/decode_trace_summary.txt
rm -f gpurun_out/prof_dec/run_kernel_trace.csv
