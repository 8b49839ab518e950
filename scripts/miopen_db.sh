#!/bin/bash
# Build a MIOpen user find-db for the n640 / n1280 / m640 backbone convs (MIOPEN_FIND_MODE=NORMAL: every applicable
# solver timed once), then check that a run reading it picks the same solvers without searching.
set -o pipefail
OUT=gpurun_out/${1:-miodb}
mkdir -p "$OUT/db"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export MIOPEN_USER_DB_PATH="$GRAFT_REPO_ROOT/$OUT/db"
for c in n640 n1280 m640; do
  MIOPEN_FIND_MODE=NORMAL timeout -k 10 400 python3 -u bench.py --config $c --no-cpu-baseline --no-nms-load --no-extra-configs \
    --steps 5 --warmup 2 > "$OUT/find_$c.json" 2> "$OUT/find_$c.err" || { tail -5 "$OUT/find_$c.err"; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' "$OUT/find_$c.json" | head -1
done
ls -la "$OUT/db"
for r in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$r" -o run -- python3 -u bench.py --no-cpu-baseline \
    --no-nms-load --no-extra-configs --steps 5 --warmup 2 > "$OUT/bench_$r.json" 2> "$OUT/bench_$r.err" || exit 1
  grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_$r.json" | head -1
  python3 - "$OUT/prof_$r" <<'PY'
import csv, sys, pathlib
f = next(pathlib.Path(sys.argv[1]).rglob("*kernel_stats.csv"))
for r in csv.DictReader(open(f)):
    if "ys::" not in r["Name"] and float(r["TotalDurationNs"]) > 1e6:
        print(f'  {int(r["Calls"]):4d} x {float(r["AverageNs"])/1e3:8.1f} us {r["Name"][:80]}')
PY
done
