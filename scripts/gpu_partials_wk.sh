# waves per workgroup of the split-K partial GEMMs (out-proj K=1024, FF-out K=4096): decode step sweep
set -o pipefail
mkdir -p gpurun_out
for wk in 2,4 1,4 2,2 2,8 1,2 4,4; do
  DALLE_AMD_PARTIALS_WK=$wk timeout -k 10 300 python3 benchmarks/bench_inference.py --batch 64 --model reference --iters 1 --no-vae > gpurun_out/inf_wk$wk.log 2>&1 || { echo "wk $wk failed"; tail -20 gpurun_out/inf_wk$wk.log; exit 1; }
  echo "wk=$wk $(grep metric gpurun_out/inf_wk$wk.log | cut -c70-250)"
done
