set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_inf -o run --output-format csv -- python3 benchmarks/bench_inference.py --batch 64 --model bench24 --profile-steps 32 > gpurun_out/prof_inf.log 2>&1 || { echo "rocprof inf failed"; tail -20 gpurun_out/prof_inf.log; exit 1; }
grep "#" gpurun_out/prof_inf.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --batch 16 > gpurun_out/prof_train.log 2>&1 || { echo "rocprof train failed"; tail -20 gpurun_out/prof_train.log; exit 1; }
tail -1 gpurun_out/prof_train.log
