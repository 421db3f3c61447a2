# per-kernel times of the attention parts at B128: text dK/dV tail split on (diag 0) / off (diag 512)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for d in 0 512; do
  DALLE_AMD_ATTN_DIAG=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/dkprof_$d -o run -- python3 benchmarks/bench_attn_parts.py 128 > gpurun_out/dkprof_$d.log 2>&1 || { echo "prof $d failed"; tail -5 gpurun_out/dkprof_$d.log; exit 1; }
  f=$(ls gpurun_out/dkprof_$d/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/dkprof_$d/run_kernel_stats.csv)
  echo "== diag=$d"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'attn' in r['Name']: print(r['Name'][:70], r['Calls'], r['AverageNs'])
"
done
