set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 benchmarks/bench_gemm.py --wgrad --m 61440 > gpurun_out/wgrad_m61440.log 2>&1 || { echo "m61440 failed"; tail -20 gpurun_out/wgrad_m61440.log; exit 1; }
grep wgrad gpurun_out/wgrad_m61440.log
timeout -k 10 300 python3 benchmarks/bench_gemm.py --wgrad --m 368640 > gpurun_out/wgrad_m368640.log 2>&1 || { echo "m368640 failed"; tail -20 gpurun_out/wgrad_m368640.log; exit 1; }
grep wgrad gpurun_out/wgrad_m368640.log
