set -o pipefail
mkdir -p gpurun_out
for parts in 2 1; do
  DALLE_AMD_DECODE_PARTS=$parts timeout -k 10 300 python3 benchmarks/decode_replay_host.py > gpurun_out/dh_$parts.log 2>&1 || { echo "failed"; tail -5 gpurun_out/dh_$parts.log; exit 1; }
  grep '^{' gpurun_out/dh_$parts.log
done
