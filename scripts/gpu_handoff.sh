# GPU check of the data-parallel gradient hand-off: fused-backward hook test, 2-rank gloo rehearsal on
# one GPU with the hand-off on and off (same loss / params), one-rank bench unchanged
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_model_gpu.py -x -v --timeout 150 --timeout-method thread -k "handoff or sequential_fused or reference_geometry" > gpurun_out/handoff_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/handoff_pytest.log; exit 1; }
tail -1 gpurun_out/handoff_pytest.log
for ov in 1 0; do
  DALLE_AMD_DP_OVERLAP=$ov BENCH_DUMP_PARAMS=gpurun_out/handoff_ov$ov BENCH_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 2 --warmup 1 --batch 8 > gpurun_out/handoff_gloo_ov$ov.log 2>&1 || { echo "2-rank gloo ov=$ov failed"; tail -30 gpurun_out/handoff_gloo_ov$ov.log; exit 1; }
  grep '^{' gpurun_out/handoff_gloo_ov$ov.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ov', $ov, d['value'], d['loss'], d.get('param_checksum'), d.get('grad_allreduce_overlapped_frac'))"
done
python3 - <<'PY'
import torch
a = [torch.load(f"gpurun_out/handoff_ov{o}.rank{r}.pt", weights_only=True) for o in (1, 0) for r in (0, 1)]
print("ranks equal (ov1, ov0):", torch.equal(a[0], a[1]), torch.equal(a[2], a[3]), "| ov1 == ov0:", torch.equal(a[0], a[2]))
PY
rm -f gpurun_out/handoff_ov*.pt
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 > gpurun_out/handoff_bench1.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/handoff_bench1.log; exit 1; }
grep '^{' gpurun_out/handoff_bench1.log | cut -c1-260
