# waves per workgroup of the split-K slab GEMMs (K < 4096, K >= 4096), two decode chains: decode step sweep
set -o pipefail
mkdir -p gpurun_out
for wk in ${WKS:-2,4 1,4 2,2 2,8 1,2 4,4}; do
  DALLE_AMD_PARTIALS_WK=$wk timeout -k 10 300 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 --no-vae > gpurun_out/inf_wk$wk.log 2>&1 || { echo "wk $wk failed"; tail -20 gpurun_out/inf_wk$wk.log; exit 1; }
  echo "wk=$wk $(grep -o '"ms_per_decode_step": [0-9.]*' gpurun_out/inf_wk$wk.log) $(grep -o '"sampling_seconds": [0-9.]*' gpurun_out/inf_wk$wk.log)"
done
