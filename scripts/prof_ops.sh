#!/bin/bash
# per-kernel times (rocprofv3 kernel trace) of bench_ops cases: bash scripts/prof_ops.sh TAG [--bf16] case...
set -o pipefail
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $OUT/p -o run -- python3 -u scripts/bench_ops.py "$@" > $OUT/out.txt 2>&1 || exit 1
grep " ms " $OUT/out.txt
python3 - $OUT/p <<'PY'
import csv, sys, pathlib
f = next(pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"))
for r in csv.DictReader(open(f)):
    if "ys::" in r["Name"]:
        print(f'  {int(r["Calls"]):4d} x {float(r["AverageNs"])/1e3:8.1f} us {r["Name"][:110]}')
PY
python3 - $OUT/p <<'PY'
import csv, sys, pathlib
f = next(pathlib.Path(sys.argv[1]).rglob("*kernel_trace.csv"))
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
rows = [r for r in rows if "ys::" in r["Kernel_Name"]]
print("last launch sequence:")
for r in rows[-12:]:
    print(f'  {(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3:8.1f} us grid {r["Grid_Size_X"]:>8s} lds {r["LDS_Block_Size"]:>6s} vgpr {r["VGPR_Count"]:>4s} {r["Kernel_Name"][:100]}')
PY
