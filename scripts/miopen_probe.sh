#!/bin/bash
# Which MIOpen solvers the backbone's stride-2 convs get on this box, with the box's user DB and with a fresh one
set -o pipefail
OUT=gpurun_out/${1:-miop}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
env | grep -i -E "miopen|rocm|hip" | sort > "$OUT/env.txt"
ls -laR ~/.config/miopen ~/.cache/miopen > "$OUT/userdb_ls.txt" 2>&1
FRESH=$(mktemp -d)
for mode in box fresh; do
  if [ $mode = fresh ]; then export MIOPEN_USER_DB_PATH=$FRESH MIOPEN_CUSTOM_CACHE_DIR=$FRESH; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$mode" -o run -- python3 -u bench.py \
    --no-cpu-baseline --no-nms-load --no-extra-configs --steps 5 --warmup 2 > "$OUT/bench_$mode.json" 2> "$OUT/bench_$mode.err" || exit 1
  python3 - "$OUT/prof_$mode" <<'PY'
import csv, sys, pathlib, json
f = next(pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"))
for r in csv.DictReader(open(f)):
    if "ys::" not in r["Name"] and float(r["TotalDurationNs"]) > 2e6:
        print(f'  {int(r["Calls"]):4d} x {float(r["AverageNs"])/1e3:8.1f} us {r["Name"][:80]}')
PY
  grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_$mode.json"
done
