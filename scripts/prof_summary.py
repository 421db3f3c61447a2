"""Summarise a rocprofv3 kernel trace: top kernels by total time.

Accepts either a ``--stats`` ``kernel_stats.csv`` (``--output-format csv``) or the default rocpd
SQLite database (``*_results.db``). ``python scripts/prof_summary.py <file> [top] [steps]``;
with ``steps`` the per-step time is printed too."""
import csv
import sqlite3
import sys
from collections import defaultdict

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 0

stats = defaultdict(lambda: [0.0, 0])  # name -> [total ns, calls]
if path.endswith(".db"):
    con = sqlite3.connect(path)
    for name, dur in con.execute("select name, duration from kernels"):
        s = stats[name]
        s[0] += float(dur)
        s[1] += 1
else:
    for r in csv.DictReader(open(path)):
        stats[r["Name"]] = [float(r["TotalDurationNs"]), int(r["Calls"])]

tot = sum(v[0] for v in stats.values())
print(f"{'total_ms':>9} {'pct':>6} {'calls':>6} {'avg_us':>8}  kernel")
for name, (ns, calls) in sorted(stats.items(), key=lambda kv: -kv[1][0])[:top]:
    print(f"{ns / 1e6:9.2f} {100 * ns / tot:6.2f} {calls:>6} {ns / calls / 1e3:8.1f}  {name[:100]}")
print(f"all kernels: {tot / 1e6:.2f} ms" + (f"  ({tot / 1e6 / steps:.2f} ms per step over {steps} steps)" if steps else ""))
