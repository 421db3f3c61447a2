# GEMM epilogue timestamps (benchmarks/gemm_epilogue_stamps.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u benchmarks/gemm_epilogue_stamps.py > gpurun_out/stamps.log 2>&1 || { echo "stamps failed"; tail -30 gpurun_out/stamps.log; exit 1; }
grep -v amdgpu.ids gpurun_out/stamps.log
