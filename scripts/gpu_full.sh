#!/bin/bash
# Full GPU pass (the one parametrised runner for a measurement set): smoke, pytest -m gpu, the default bench line
# (compact stdout line + its detail file + the per-launch CSV), then the rocprofv3 kernel summary of the headline
# config (its own process). Results under gpurun_out/TAG; copy what is judged into profiles/.
#   bash scripts/gpu_full.sh TAG [--no-tests]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
rc=0
if [ "$2" != "--no-tests" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "smoke failed"; tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.log" 2>&1
  rc=$?
  grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -15
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --detail-json "$OUT/bench_detail.json" \
  --ops-csv "$OUT/ops_calls.csv" > "$OUT/bench.json" 2> "$OUT/bench.err" \
  || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
wc -c "$OUT/bench.json"
cut -c1-400 "$OUT/bench.json"
python3 scripts/roofline_from_csv.py "$OUT/ops_calls.csv" "$OUT/bench_detail.json" > "$OUT/recompute.txt" 2>&1
tail -1 "$OUT/recompute.txt"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py \
  --steps 20 --warmup 5 --no-cpu-baseline --no-nms-load --no-extra-configs --detail-json "$OUT/prof_detail.json" \
  > "$OUT/bench_rocprof.json" 2> "$OUT/bench_rocprof.err" || { echo "rocprof failed"; tail -5 "$OUT/bench_rocprof.err"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" | head -3
exit $rc
