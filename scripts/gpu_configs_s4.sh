set -o pipefail
# every BASELINE config on one MI355X (bench24 step + collab engine, PowerSGD, reference recipe, 1.3B, inference)
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python3 bench.py "$@" --profile-steps 2 > gpurun_out/cfg_r2s4_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/cfg_r2s4_$name.log; exit 1; }
  grep -h "metric\|phase" gpurun_out/cfg_r2s4_$name.log | cut -c1-300
}
run step 240 --steps 10 --warmup 3
run collab 240 --steps 10 --warmup 3 --engine collab
run psgd8 240 --steps 5 --warmup 2 --compression powersgd --optim-bits 8
run ref48_recompute 400 --model reference --batch 48 --steps 3 --warmup 1 --recompute true
run ref48_auto 400 --model reference --batch 48 --steps 3 --warmup 1 --recompute auto
run l13_32_recompute 400 --model dalle-1.3b --batch 32 --steps 3 --warmup 1 --recompute true
run l13_32_auto 400 --model dalle-1.3b --batch 32 --steps 3 --warmup 1 --recompute auto
timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model bench24 --iters 2 > gpurun_out/cfg_r2s4_inf24.log 2>&1 || { echo "inf24 failed"; tail -20 gpurun_out/cfg_r2s4_inf24.log; exit 1; }
grep metric gpurun_out/cfg_r2s4_inf24.log | cut -c1-300
timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 2 > gpurun_out/cfg_r2s4_infref.log 2>&1 || { echo "infref failed"; tail -20 gpurun_out/cfg_r2s4_infref.log; exit 1; }
grep metric gpurun_out/cfg_r2s4_infref.log | cut -c1-300
# data-parallel hand-off on the unshared 1.3B reversible preset: 2-rank gloo rehearsal on this one GPU
BENCH_BACKEND=gloo timeout -k 10 400 python3 bench.py --model dalle-1.3b --gpus 2 --steps 2 --warmup 1 --batch 2 --recompute true > gpurun_out/cfg_r2s4_l13_gloo2.log 2>&1 || { echo "1.3b gloo failed"; tail -30 gpurun_out/cfg_r2s4_l13_gloo2.log; exit 1; }
grep -h metric gpurun_out/cfg_r2s4_l13_gloo2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('l13 gloo2', d['n_gpus'], d['loss'], 'overlapped_frac', d.get('grad_allreduce_overlapped_frac'))"
