# round 6: repeated-caption decode, run-to-run check (the flag per part in the JSON line)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in "" --same-caption "" --same-caption; do
  timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --iters 3 $c > gpurun_out/r6t_inf2.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r6t_inf2.log; exit 1; }
  echo "caption=${c:-distinct} $(grep -h '^{' gpurun_out/r6t_inf2.log | grep -o '"value": [0-9.]*\|"ms_per_decode_step": [0-9.]*\|"text_shared": \[[0-9, ]*\]' | tr '\n' ' ')"
done
