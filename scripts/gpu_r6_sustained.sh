# round 6: sustained runs -- does the short bench's number hold over minutes at the board's power limit?
# bench24 over 200 timed steps (~80 s) and generation over 6 batches, with rocm-smi power / clock samples alongside
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
sample() {  # $1: output file; samples every 5 s until the marker file disappears
  touch gpurun_out/.sampling
  while [ -e gpurun_out/.sampling ]; do
    { date +%s; timeout 10 rocm-smi --showpower --showclocks --showtemp 2>&1 | grep -E "Power|sclk|mclk|Temperature" ; } >> "$1"
    sleep 5
  done
}
sample gpurun_out/r6s_smi_train.log &
SP=$!
timeout -k 10 400 python3 bench.py --steps 200 --warmup 5 > gpurun_out/r6s_bench.log 2>&1
RC=$?
rm -f gpurun_out/.sampling
wait $SP
[ $RC -eq 0 ] || { echo "bench failed rc=$RC"; tail -20 gpurun_out/r6s_bench.log; exit 1; }
grep '^{' gpurun_out/r6s_bench.log | cut -c1-400
sample gpurun_out/r6s_smi_gen.log &
SP=$!
timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --iters 6 --same-caption > gpurun_out/r6s_gen.log 2>&1
RC=$?
rm -f gpurun_out/.sampling
wait $SP
[ $RC -eq 0 ] || { echo "generation failed rc=$RC"; tail -20 gpurun_out/r6s_gen.log; exit 1; }
grep -E '^#|^\{' gpurun_out/r6s_gen.log | cut -c1-400
