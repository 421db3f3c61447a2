# TunableOp (hipBLASLt / rocBLAS per-shape solution search) on the bench24 micro-batch-128 step: tune once,
# then alternate use / off on the same box. The tuned CSV is copied to gpurun_out/ for inspection.
set -o pipefail
mkdir -p gpurun_out
rm -f profiles/tunableop_gfx950.csv
timeout -k 10 900 python3 bench.py --steps 2 --warmup 1 --tunable tune > gpurun_out/tun_tune.log 2>&1 || { echo "tune failed"; tail -20 gpurun_out/tun_tune.log; exit 1; }
grep '^{' gpurun_out/tun_tune.log | cut -c1-200
cp profiles/tunableop_gfx950.csv gpurun_out/tunableop_gfx950_b128.csv 2>/dev/null; wc -l gpurun_out/tunableop_gfx950_b128.csv
for m in use off use off; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --tunable $m > gpurun_out/tun_$m.log 2>&1 || { echo "$m failed"; tail -20 gpurun_out/tun_$m.log; exit 1; }
  echo "$m $(grep '^{' gpurun_out/tun_$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["config"].get("gemm_selection"))')"
done
