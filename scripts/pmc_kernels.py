"""Per-kernel HBM bytes per dispatch from scripts/pmc_run.sh output (FETCH_SIZE x2 gfx950 read correction +
WRITE_SIZE, KiB -> MB): python scripts/pmc_kernels.py OUTDIR case"""
import collections
import csv
import sys
from pathlib import Path

out, case = Path(sys.argv[1]), sys.argv[2]
rows = collections.defaultdict(lambda: [0.0, 0.0, set()])
for kind, counter in (("f", "FETCH_SIZE"), ("w", "WRITE_SIZE")):
    for f in (out / f"{case}_{kind}").rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter or not r["Kernel_Name"].startswith(("ys::", "void ys::")):
                continue
            k = r["Kernel_Name"][:80]
            rows[k][0 if kind == "f" else 1] += float(r["Counter_Value"])
            rows[k][2].add((kind, r["Dispatch_Id"]))
tot = 0.0
for k, (fs, ws, d) in sorted(rows.items()):
    n = max(1, len([x for x in d if x[0] == "f"]))
    rd, wr = 2 * fs / n / 1024, ws / max(1, len([x for x in d if x[0] == "w"])) / 1024
    tot += rd + wr
    print(f"{k:80s} read {rd:8.2f} MB  write {wr:8.2f} MB")
print(f"total per call {tot:.1f} MB")
