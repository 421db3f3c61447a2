# round 6: with per-part linear graphs (host ~0.2 ms per graph launch), are 4 quarter-batch chains better than 2?
# (round 2 measured 4 parts at 4.0-6.1 ms per step, but through the node-by-node joint graph)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for parts in 4 2; do
  DALLE_AMD_DECODE_PARTS=$parts timeout -k 10 240 python3 benchmarks/probe_replay_host.py > gpurun_out/r6p4_probe_$parts.log 2>&1 || { echo "probe $parts failed"; tail -5 gpurun_out/r6p4_probe_$parts.log; exit 1; }
  echo "probe parts=$parts $(grep '^{' gpurun_out/r6p4_probe_$parts.log)"
done
for rep in 1 2; do
  for parts in 4 2; do
    for cap in "--same-caption" ""; do
      DALLE_AMD_DECODE_PARTS=$parts timeout -k 10 300 python3 benchmarks/bench_inference.py --batch 64 --iters 4 $cap > gpurun_out/r6p4_gen.log 2>&1 || { echo "gen $parts $cap failed"; tail -5 gpurun_out/r6p4_gen.log; exit 1; }
      echo "gen parts=$parts cap=${cap:-distinct} $(grep -E '^# generate' gpurun_out/r6p4_gen.log | tr '\n' ' ') $(grep '^{' gpurun_out/r6p4_gen.log | grep -oE '"value": [0-9.]+|"ms_per_decode_step": [0-9.]+|"sampling_seconds": [0-9.]+|"decode_parts": [0-9]+' | tr '\n' ' ')"
    done
  done
done
