#!/bin/bash
# round 4: ablations of the token-tiled MLP kernel (timing only; the ablated builds compute wrong results)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04c; mkdir -p $O
for lib in "" ab4/lib_TOKMEM.so ab4/lib_TOKT1.so ab4/lib_TOKMEM_T1.so; do
  n=$(basename "${lib:-base}" .so)
  YOLOSOD_LIB_AB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/$n -o run -- python3 -u scripts/bench_ops.py swin_L28 > $O/$n.txt 2>&1 || exit 1
  python3 - $O/$n $n <<'PY'
import csv, sys, pathlib
f = next(pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"))
for r in csv.DictReader(open(f)):
    if "ys::" in r["Name"]:
        print(f'{sys.argv[2]:14s} {int(r["Calls"]):4d} x {float(r["AverageNs"])/1e3:8.1f} us {r["Name"][:80]}')
PY
done
