#!/bin/bash
# per-kernel times of the A2 launch sequence for the in-tree build and the ab_push/ diagnostic builds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-profa2}; mkdir -p $OUT
for lib in "" $(ls ab_push/*.so); do
  tag=$(basename ${lib:-tree} .so)
  YOLOSOD_LIB_AB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $OUT/$tag -o run -- python3 -u scripts/bench_ops.py ${CASES:-a2_L12} > $OUT/$tag.txt 2>&1 || exit 1
  echo "== $tag"; grep " ms " $OUT/$tag.txt
  python3 - $OUT/$tag <<'PY'
import csv, sys, pathlib
f = next(pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"))
for r in csv.DictReader(open(f)):
    if "ys::" in r["Name"]:
        print(f'  {int(r["Calls"]):4d} x {float(r["AverageNs"])/1e3:8.1f} us {r["Name"][:90]}')
PY
done
