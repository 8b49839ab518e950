#!/bin/bash
# Per-kernel NMS time at fixed loads (B=32, A=34000, nc=10, predict mode): bench_nms.py wall time, then one
# rocprofv3 kernel summary per load. bash scripts/nms_prof.sh TAG [loads...]  (results under gpurun_out/TAG)
set -o pipefail
TAG=$1; shift
LOADS=${*:-0 1000 10000 30000}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u scripts/bench_nms.py $LOADS > "$OUT/bench_nms.txt" 2>&1 || exit $?
cat "$OUT/bench_nms.txt"
for n in $LOADS; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/prof_$n" -o run -- python3 scripts/bench_nms.py $n \
    > "$OUT/prof_$n.log" 2>&1 || exit $?
  f=$(find "$OUT/prof_$n" -name '*kernel_stats.csv' | head -1)
  if [ -n "$f" ]; then cp "$f" "$OUT/kernel_stats_$n.csv"; echo "== $n"; grep -i "nms" "$OUT/kernel_stats_$n.csv" | cut -d, -f1-5; fi
  find "$OUT/prof_$n" -type f ! -name '*stats.csv' -delete
done
exit 0
