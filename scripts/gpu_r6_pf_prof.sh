# round 6: kernel statistics of the distinct-caption prefill (5 calls of the split engine's prefill, batch 64)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 200 python3 benchmarks/bench_prefill.py > gpurun_out/pf_plain.log 2>&1 || { echo "prefill failed"; tail -5 gpurun_out/pf_plain.log; exit 1; }
cat gpurun_out/pf_plain.log | grep '^{'
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_pf -o run --output-format csv -- python3 $R/benchmarks/bench_prefill.py > $R/gpurun_out/prof_pf.log 2>&1 || { echo "prof failed"; tail -20 $R/gpurun_out/prof_pf.log; exit 1; }
cd $R
rm -f gpurun_out/prof_pf/run_kernel_trace.csv
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open("gpurun_out/prof_pf/run_kernel_stats.csv")))
tot=sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms over 5 prefills + 1 capture warm-up")
for r in sorted(rows,key=lambda r:-float(r["TotalDurationNs"]))[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:8.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:110]}')
PY
