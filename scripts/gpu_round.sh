#!/bin/bash
# GPU box pass: full -m gpu suite, then bench lines for the given configs (default n640 m640).
# Usage: bash scripts/gpu_round.sh TAG [configs...]
set -o pipefail
TAG=${1:-run}
shift
CONFIGS=${@:-n640 m640}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (keep benching); anything else = stop
for c in $CONFIGS; do
  timeout -k 10 400 python -u bench.py --config $c > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || { echo "bench $c failed"; tail -20 "$OUT/bench_$c.err"; exit 1; }
  cut -c1-600 "$OUT/bench_$c.json"
done
exit $rc
