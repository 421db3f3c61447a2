# text dK/dV workgroup shape A/B: KBW key blocks per workgroup (2 or 3) x occupancy variant; attention tests with the default
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kb_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/kb_pytest.log; exit 1; }
tail -1 gpurun_out/kb_pytest.log
for cfg in "2 3,3,2,2" "3 3,3,2,2" "3 3,3,3,2" "2 3,3,2,2"; do
  set -- $cfg
  DALLE_AMD_DKDV_KB=$1 DALLE_AMD_ATTN_OCC=$2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kb_$1_$2 -o run --output-format csv -- python3 benchmarks/attn_bwd_diag.py > gpurun_out/kb_$1_$2.log 2>&1 || { echo "prof failed $cfg"; tail -5 gpurun_out/kb_$1_$2.log; exit 1; }
  echo "KB=$1 OCC=$2: $(grep -h dkdv_text gpurun_out/kb_$1_$2/run_kernel_stats.csv | awk -F, '{print $2, $3, $4}' | head -2)"
  rm -f gpurun_out/kb_$1_$2/run_kernel_trace.csv
done
