#!/bin/bash
# rocprofv3 kernel summary of scripts/bench_ops.py cases: bash scripts/prof_ops.sh TAG [--bf16] case...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof" -o run -- python3 -u scripts/bench_ops.py "$@" \
  > "$OUT/ops.txt" 2> "$OUT/ops.err" || { echo "rocprof failed"; tail -20 "$OUT/ops.err"; exit 1; }
cat "$OUT/ops.txt"
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1)
cp "$f" "$OUT/kernel_stats.csv"
python3 - "$OUT/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):5d} x {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:100]}')
PY
