"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels by total time."""
import csv
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'total_ms':>9} {'pct':>6} {'calls':>6} {'avg_us':>8}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} {float(r['Percentage']):6.2f} {r['Calls']:>6} {float(r['AverageNs'])/1e3:8.1f}  {r['Name'][:100]}")
print(f"all kernels: {tot/1e6:.2f} ms")
