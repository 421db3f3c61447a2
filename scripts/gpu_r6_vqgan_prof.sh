# round 6: VQGAN decoder (batch 64) kernel statistics on the HIP path
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 200 python3 benchmarks/bench_vqgan.py --iters 3 > gpurun_out/vq_plain.log 2>&1 || { echo "vqgan failed"; tail -5 gpurun_out/vq_plain.log; exit 1; }
grep '^{' gpurun_out/vq_plain.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_vq -o run --output-format csv -- python3 $R/benchmarks/bench_vqgan.py --iters 3 > $R/gpurun_out/prof_vq.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_vq.log; exit 1; }
cd $R
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open("gpurun_out/prof_vq/run_kernel_trace.csv")))
# HIP-path kernels only: the conv / GN / upsample kernels of dalle::, grouped by name and grid
from collections import defaultdict
agg=defaultdict(lambda:[0,0.0])
for r in rows:
    n=r["Kernel_Name"]
    if "dalle::" not in n: continue
    key=(n[:90], r.get("Grid_Size_X",""), r.get("Grid_Size_Y",""), r.get("Grid_Size_Z",""), r.get("Workgroup_Size_X",""))
    agg[key][0]+=1; agg[key][1]+=(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3
tot=sum(v[1] for v in agg.values())
print(f"dalle:: kernels total {tot/1e3:.1f} ms")
for k,v in sorted(agg.items(), key=lambda kv:-kv[1][1])[:30]:
    print(f"{v[1]/1e3:8.2f} ms {v[0]:5d} calls {v[1]/v[0]:9.1f} us grid={k[1]}x{k[2]}x{k[3]} wg={k[4]}  {k[0]}")
PY
rm -f gpurun_out/prof_vq/run_kernel_trace.csv
