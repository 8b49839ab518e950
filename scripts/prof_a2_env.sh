#!/bin/bash
# per-kernel times of the A2 launch sequence under GEMM tile overrides (YOLOSOD_GEMM_TILE)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-profa2e}; mkdir -p $OUT
for t in 0 1 2 3; do
  YOLOSOD_GEMM_TILE=$t timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/t$t -o run -- python3 -u scripts/bench_ops.py a2_L12 > $OUT/t$t.txt 2>&1 || exit 1
  echo "== tile $t"; grep " ms " $OUT/t$t.txt
  python3 - $OUT/t$t <<'PY'
import csv, sys, pathlib
f = next(pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"))
for r in csv.DictReader(open(f)):
    if "gemm" in r["Name"]:
        print(f'  {int(r["Calls"]):4d} x {float(r["AverageNs"])/1e3:8.1f} us {r["Name"][:90]}')
PY
done
