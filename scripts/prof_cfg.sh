#!/bin/bash
# rocprofv3 kernel summary of one bench config: bash scripts/prof_cfg.sh TAG CONFIG [extra bench args]
set -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$CFG" -o run -- python3 -u bench.py --config $CFG \
  --no-cpu-baseline --no-nms-load "$@" > "$OUT/bench_${CFG}_rocprof.json" 2> "$OUT/bench_${CFG}_rocprof.err" || { echo "rocprof failed"; tail -20 "$OUT/bench_${CFG}_rocprof.err"; exit 1; }
f=$(find "$OUT/prof_$CFG" -name '*kernel_stats.csv' | head -1)
cp "$f" "$OUT/kernel_stats_$CFG.csv"
python3 - "$OUT/kernel_stats_$CFG.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms")
for r in rows[:30]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):5d} x {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
