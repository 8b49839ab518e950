#!/bin/bash
# r03 session: tests touched by the split2 change + new parity tests, then op A/B vs ablib/lib_prev.so, then bench
set -o pipefail
TAG=${1:-r03b}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 600 python -u -m pytest tests/test_gpu_split_range.py tests/test_gpu_e2e.py tests/test_gpu_ops.py tests/test_gpu_model.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  echo "-- A prev"; YOLOSOD_LIB_AB=ablib/lib_prev.so timeout -k 10 120 python -u scripts/bench_ops.py swin_L28 swin_L9 a2_L12 head 2>&1 | grep " ms " || exit 1
  echo "-- B cur"; timeout -k 10 120 python -u scripts/bench_ops.py swin_L28 swin_L9 a2_L12 head 2>&1 | grep " ms " || exit 1
done
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
cut -c1-400 "$OUT/bench.json"
exit $rc
