# decode split-K partial modes (0: in-GEMM hand-off, 1: residual projections as slabs summed by the next
# LayerNorm, 2: + QKV slabs summed in the attention prologue): generation GPU tests, then same-box A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_generation_gpu.py tests/test_skinny_gpu.py > gpurun_out/part_tests.log 2>&1 || { tail -40 gpurun_out/part_tests.log; exit 1; }
tail -1 gpurun_out/part_tests.log
for v in ${MODES:-0 1 2}; do
  DALLE_AMD_DECODE_PARTIALS=$v timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 > gpurun_out/inf_part$v.log 2>&1 || { echo "inference $v failed"; tail -20 gpurun_out/inf_part$v.log; exit 1; }
  echo "partials=$v $(grep metric gpurun_out/inf_part$v.log | cut -c70-330)"
done
P=${PROF:-1}
DALLE_AMD_DECODE_PARTIALS=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dp$P -o run --output-format csv -- python3 benchmarks/bench_inference.py --batch 64 --model reference --profile-steps 64 --no-vae > gpurun_out/prof_dp$P.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_dp$P.log; exit 1; }
rm -f gpurun_out/prof_dp$P/run_kernel_trace.csv
python3 scripts/prof_summary.py gpurun_out/prof_dp$P/run_kernel_stats.csv 12 1 > gpurun_out/prof_dp${P}_top.txt
head -10 gpurun_out/prof_dp${P}_top.txt | cut -c1-140
