"""Per-step kernel-time summary of a ``rocprofv3 --kernel-trace --stats`` run of bench.py.

    python benchmarks/kernel_stats.py <rocprofv3 output dir> <steps profiled (warmup + timed)> [--top 30]

Reads every ``*kernel_stats.csv`` (CSV output) or rocpd ``*.db`` (the default SQLite output) under the directory and prints ms/step, share, calls/step and the mean
duration per kernel, plus the hipBLASLt (Cijk_*) share of the step."""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("steps", type=int)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = {}
    for path in glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True):   # rocpd SQLite output
        import sqlite3
        con = sqlite3.connect(path)
        for name, calls, total in con.execute("select name, count(*), sum(duration) from kernels group by name"):
            c0, t0 = rows.get(name, (0, 0.0))
            rows[name] = (c0 + calls, t0 + float(total))
    for path in glob.glob(os.path.join(a.dir, "**", "*kernel_stats.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                name = r["Name"]
                calls, total = int(r["Calls"]), float(r["TotalDurationNs"])
                c0, t0 = rows.get(name, (0, 0.0))
                rows[name] = (c0 + calls, t0 + total)
    total = sum(t for _, t in rows.values())
    cijk = sum(t for n, (_, t) in rows.items() if n.startswith(("Cijk", "Custom_Cijk")))
    print(f"# total GPU time {total / 1e6 / a.steps:.1f} ms/step; Cijk (hipBLASLt) share {100 * cijk / max(total, 1):.1f} %")
    for name, (calls, t) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{t / 1e6 / a.steps:8.2f} ms/step {100 * t / total:5.1f}% calls/step={calls / a.steps:5.1f} "
              f"avg={t / 1e3 / max(calls, 1):9.1f}us {name[:140]}")


if __name__ == "__main__":
    main()
