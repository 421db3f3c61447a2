# persistent-GEMM epilogue cost vs concurrent storers, then the full round-3 GPU check (tests, smoke, benches, rocprof)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u benchmarks/gemm_epilogue_grid.py > gpurun_out/grid.log 2>&1 || { echo "grid failed"; tail -30 gpurun_out/grid.log; exit 1; }
grep -v amdgpu.ids gpurun_out/grid.log
bash scripts/gpu_check3.sh r3s2
