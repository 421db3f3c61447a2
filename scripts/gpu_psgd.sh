set -o pipefail
# PowerSGD kernels: numerics, config-3 throughput; kernel profile of the reference recipe (reversible)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_powersgd_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_psgd.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_psgd.log; exit 1; }
tail -2 gpurun_out/pytest_psgd.log
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --compression powersgd --optim-bits 8 --profile-steps 2 > gpurun_out/cfg_psgd8.log 2>&1 || { echo "psgd bench failed"; tail -30 gpurun_out/cfg_psgd8.log; exit 1; }
grep -h "metric\|phase" gpurun_out/cfg_psgd8.log | cut -c1-120,400-900
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_ref -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model reference --batch 48 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_ref.log 2>&1 || { echo "rocprof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_ref.log; exit 1; }
echo done
