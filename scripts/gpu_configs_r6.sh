set -o pipefail
# every BASELINE config on one MI355X at the round-6 defaults (micro-batch variants of the large configs; generation with a
# distinct caption per row and with one caption repeated over the batch, as inference/run_inference.py generates)
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python3 bench.py "$@" > gpurun_out/cfg_r6_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/cfg_r6_$name.log; exit 1; }
  echo "$name $(grep -h '^{' gpurun_out/cfg_r6_$name.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('max_mem_gb'), d['config'].get('per_gpu_batch'))")"
}
run step128 300 --steps 10 --warmup 3
run collab 300 --steps 10 --warmup 3 --engine collab
run psgd8 300 --steps 5 --warmup 2 --compression powersgd --optim-bits 8
run ref48_recompute 400 --model reference --batch 48 --steps 3 --warmup 1 --recompute true
run ref48_auto 400 --model reference --batch 48 --steps 3 --warmup 1 --recompute auto
run l13_32_auto 400 --model dalle-1.3b --batch 32 --steps 3 --warmup 1 --recompute auto
timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 2 > gpurun_out/cfg_r6_infref.log 2>&1 || { echo "infref failed"; tail -20 gpurun_out/cfg_r6_infref.log; exit 1; }
grep metric gpurun_out/cfg_r6_infref.log | cut -c1-200
timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 2 --same-caption > gpurun_out/cfg_r6_infref_same.log 2>&1 || { echo "infref same failed"; tail -20 gpurun_out/cfg_r6_infref_same.log; exit 1; }
grep metric gpurun_out/cfg_r6_infref_same.log | cut -c1-200
