# skinny decode GEMMs: default vs wave -> K-chunk map rotated per column tile (dbg 8, 12 = + permuted K order)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 benchmarks/bench_skinny.py --batch 64 --rotate --ablate > gpurun_out/skinny_rotate.jsonl 2>&1 || { tail -20 gpurun_out/skinny_rotate.jsonl; exit 1; }
grep '^{' gpurun_out/skinny_rotate.jsonl | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['op'], d['nbv_wk_ks_steps_dbg'], d['skinny_us'], d['hipblaslt_us'])"
