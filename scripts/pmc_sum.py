"""Per-kernel mean of every counter in rocprofv3 --pmc counter_collection CSVs (one or more passes):
    python scripts/pmc_sum.py DIR [kernel-substring]"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root, sub = Path(sys.argv[1]), (sys.argv[2] if len(sys.argv) > 2 else "")
vals = defaultdict(lambda: defaultdict(list))
for f in root.rglob("*counter_collection.csv"):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            per[(r["Kernel_Name"].split("(")[0][-60:], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (k, _, c), v in per.items():
        vals[k][c].append(v)
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
