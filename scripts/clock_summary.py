"""Effective clock per kernel from scripts/clock_run.sh output: GRBM_GUI_ACTIVE / 8 XCDs / kernel duration.

usage: python scripts/clock_summary.py OUTDIR"""
import collections
import csv
import sys
from pathlib import Path

out = Path(sys.argv[1])
for f in sorted(out.rglob("*counter_collection.csv")):
    case = f.relative_to(out).parts[0]
    act = collections.defaultdict(float)
    name = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            act[r["Dispatch_Id"]] += float(r["Counter_Value"])
            name[r["Dispatch_Id"]] = r["Kernel_Name"]
    dur = {}
    for t in f.parent.rglob("*kernel_trace.csv"):
        for r in csv.DictReader(open(t)):
            dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    per = collections.defaultdict(list)
    for d, a in act.items():
        if d in dur and dur[d] > 0 and name[d].startswith(("ys::", "void ys::")):
            per[name[d][:70]].append((a / 8.0 / dur[d] / 1e9, dur[d] * 1e3))
    for k, v in per.items():
        v = v[len(v) // 2:]  # second half: warm
        print(f"{case:16s} {k:70s} clock {sum(c for c, _ in v) / len(v):.3f} GHz  ({sum(t for _, t in v) / len(v):.3f} ms, n={len(v)})")
