# round 6: the two decode chains on disjoint CU sets (CU-masked streams) vs sharing all CUs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in "" block interleave; do
  DALLE_AMD_DECODE_CU_SPLIT=$mode timeout -k 10 240 python3 benchmarks/probe_replay_host.py > gpurun_out/r6cu_probe.log 2>&1 || { echo "probe $mode failed"; tail -5 gpurun_out/r6cu_probe.log; exit 1; }
  echo "probe split=${mode:-none} $(grep '^{' gpurun_out/r6cu_probe.log | grep -oE '"256": \{[^}]*\}|"event_ms_per_step": [0-9.]+')"
done
for rep in 1 2; do
  for mode in "" block interleave; do
    for cap in "--same-caption" ""; do
      DALLE_AMD_DECODE_CU_SPLIT=$mode timeout -k 10 300 python3 benchmarks/bench_inference.py --batch 64 --iters 3 $cap > gpurun_out/r6cu_gen.log 2>&1 || { echo "gen $mode $cap failed"; tail -5 gpurun_out/r6cu_gen.log; exit 1; }
      echo "gen split=${mode:-none} cap=${cap:-distinct} $(grep -E '^# batched' gpurun_out/r6cu_gen.log | tr '\n' ' ') $(grep '^{' gpurun_out/r6cu_gen.log | grep -oE '"value": [0-9.]+|"ms_per_decode_step": [0-9.]+|"sampling_seconds": [0-9.]+' | tr '\n' ' ')"
    done
  done
done
