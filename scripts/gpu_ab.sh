#!/bin/bash
# GPU tests (pytest args in T, e.g. T="tests/test_gpu_ops.py -k swin") + same-box A/B of bench_ops cases between a
# library build A (ab_push/*.so) and the current build: bash scripts/gpu_ab.sh TAG LIB_A case [case ...]
set -o pipefail
TAG=$1; A=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
if [ -n "$T" ]; then
  timeout -k 10 600 python -u -m pytest $T -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -12
  [ $rc -eq 0 ] || [ $rc -eq 5 ] || [ $rc -eq 1 ] || exit $rc
fi
for r in 1 2; do
  echo "-- A ($A)"; YOLOSOD_LIB_AB=$A timeout -k 10 120 python -u scripts/bench_ops.py "$@" 2>&1 | grep " ms " || exit 1
  echo "-- B (current)"; timeout -k 10 120 python -u scripts/bench_ops.py "$@" 2>&1 | grep " ms " || exit 1
done
