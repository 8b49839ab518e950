"""Per-kernel SQ counter summary of scripts/sq_run.sh output: python scripts/sq_summary.py OUTDIR."""
import collections
import csv
import sys
from pathlib import Path

out = Path(sys.argv[1])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for f in sorted(out.rglob("*counter_collection.csv")):
    case = f.relative_to(out).parts[0].rsplit("_", 1)[0]
    for r in csv.DictReader(open(f)):
        k = (case, r["Kernel_Name"][:70])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add(r["Dispatch_Id"])
for (case, kern), c in sorted(agg.items()):
    if not kern.startswith(("ys::", "void ys::")):
        continue
    n = max(len(calls[(case, kern)]), 1)
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{case:12s} {kern}")
    print("   " + "  ".join(f"{k[3:]}={v / n:.4g}" for k, v in sorted(c.items())))
    if "SQ_WAIT_ANY" in c:
        print(f"   shares of wave cycles: active {c['SQ_ACTIVE_INST_ANY'] / wc:.2f} wait {c['SQ_WAIT_ANY'] / wc:.2f} "
              f"wait_inst {c['SQ_WAIT_INST_ANY'] / wc:.2f}; mfma_busy/busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(c['SQ_BUSY_CYCLES'], 1):.3g}")
