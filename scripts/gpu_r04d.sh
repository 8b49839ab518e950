#!/bin/bash
# round 4: memory-behaviour variants of the token-tiled MLP kernel (YS_TOK_DIAG bits; timing only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04d; mkdir -p $O
for d in 0 1 2 4 8 12 16 28; do
  YS_TOK_DIAG=$d timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/d$d -o run -- python3 -u scripts/bench_ops.py swin_L28 > $O/d$d.txt 2>&1 || exit 1
  python3 - $O/d$d $d <<'PY'
import csv, sys, pathlib
f = next(pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"))
for r in csv.DictReader(open(f)):
    if "ys::" in r["Name"] and "prep" not in r["Name"]:
        print(f'diag {sys.argv[2]:3s} {int(r["Calls"]):4d} x {float(r["AverageNs"])/1e3:8.1f} us {r["Name"][:70]}')
PY
done
