set -o pipefail
# every BASELINE config on one MI355X (bench24 step + collab engine, PowerSGD, reference recipe, 1.3B, inference)
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python3 bench.py "$@" --profile-steps 2 > gpurun_out/cfg_r2_$name.log 2>&1 || { echo "$name failed"; tail -30 gpurun_out/cfg_r2_$name.log; exit 1; }
  grep -h "metric\|phase" gpurun_out/cfg_r2_$name.log | cut -c1-300
}
run psgd8 240 --steps 5 --warmup 2 --compression powersgd --optim-bits 8
run ref48_recompute 400 --model reference --batch 48 --steps 3 --warmup 1 --recompute true
run ref48_auto 400 --model reference --batch 48 --steps 3 --warmup 1 --recompute auto
run l13_32_recompute 400 --model dalle-1.3b --batch 32 --steps 3 --warmup 1 --recompute true
run l13_32_auto 400 --model dalle-1.3b --batch 32 --steps 3 --warmup 1 --recompute auto
timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model bench24 --iters 2 > gpurun_out/cfg_r2_inf24.log 2>&1 || { echo "inf24 failed"; tail -20 gpurun_out/cfg_r2_inf24.log; exit 1; }
grep metric gpurun_out/cfg_r2_inf24.log | cut -c1-300
timeout -k 10 400 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 2 > gpurun_out/cfg_r2_infref.log 2>&1 || { echo "infref failed"; tail -20 gpurun_out/cfg_r2_infref.log; exit 1; }
grep metric gpurun_out/cfg_r2_infref.log | cut -c1-300
