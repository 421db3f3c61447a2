"""Raw per-kernel means of every counter in rocprofv3 --pmc csv passes: python scripts/pmc_raw.py DIR [DIR ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            name = r.get("Kernel_Name", "?")[:60]
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in vals.items():
    if "attn" not in name and "dalle" not in name:
        continue
    print(name)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} mean {sum(v) / len(v):16.1f}  (n={len(v)})")
