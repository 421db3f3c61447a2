# bench.py A/B on one box: head chunk 16384 (default) vs 32768 rows, alternating A B A B
mkdir -p gpurun_out
: > gpurun_out/head_chunk_ab.txt
for i in 1 2; do
  for c in 16384 32768; do
    DALLE_AMD_HEAD_CHUNK_ROWS=$c timeout -k 10 300 python3 bench.py --steps 15 > gpurun_out/hc_$c.log 2>&1 || exit 1
    echo "$c $(grep -h '^{' gpurun_out/hc_$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/head_chunk_ab.txt
  done
done
