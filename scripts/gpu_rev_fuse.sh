# reversible stack: residual update fused with the next LayerNorm (ln_shift_fwd_res) vs separate kernels
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_train_gpu.py tests/test_model_gpu.py tests/test_fused_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/rev_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/rev_pytest.log; exit 1; }
tail -1 gpurun_out/rev_pytest.log
for rep in 1 2; do
for f in 1 0; do
  DALLE_AMD_FUSED_SEQUENTIAL=$f timeout -k 10 300 python3 bench.py --model reference --batch 48 --recompute auto --steps 5 --warmup 2 > gpurun_out/rev_ref_$f.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/rev_ref_$f.log; exit 1; }
  echo "reference auto fused=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rev_ref_$f.log)"
  DALLE_AMD_FUSED_SEQUENTIAL=$f timeout -k 10 300 python3 bench.py --model dalle-1.3b --batch 32 --steps 4 --warmup 2 > gpurun_out/rev_13_$f.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/rev_13_$f.log; exit 1; }
  echo "1.3b rebuild fused=$f $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/rev_13_$f.log)"
done
done
