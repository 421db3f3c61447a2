set -o pipefail
mkdir -p gpurun_out
DALLE_AMD_ATTN_BWD_CONC=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or rotary or axial" > gpurun_out/conc_tests.log 2>&1 || { tail -30 gpurun_out/conc_tests.log; exit 1; }
tail -1 gpurun_out/conc_tests.log
bash scripts/gpu_ab.sh DALLE_AMD_ATTN_BWD_CONC 0 1
