#!/bin/bash
# Full GPU pass: pytest -m gpu, then the bench line, then the rocprofv3 kernel summary of the same bench command
# (kept under profiles/ by the caller). Usage: bash scripts/gpu_full.sh TAG
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-300 "$OUT/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-nms-load --no-extra-configs > "$OUT/bench_rocprof.json" 2> "$OUT/bench_rocprof.err" || { echo "rocprof failed"; tail -5 "$OUT/bench_rocprof.err"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" | head -3
exit $rc
