# round 6: LDS-tiled RGB output conv of the VQGAN decoder: kernel + decoder tests, then the decoder kernel statistics
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_vqgan_gpu.py tests/test_generation_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6co_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r6co_pytest.log | head -30; tail -30 gpurun_out/r6co_pytest.log; exit 1; }
tail -1 gpurun_out/r6co_pytest.log
bash scripts/gpu_r6_vqgan_prof.sh
