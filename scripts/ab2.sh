#!/bin/bash
# GPU tests (pytest -k EXPR) on library B, then same-box A/B timing: bash scripts/ab2.sh TAG "expr" LIB_A LIB_B case...
# (LIB_* = "" for the in-tree build)
set -o pipefail
TAG=$1; K=$2; A=$3; B=$4; shift 4
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
YOLOSOD_LIB_AB=$B timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_split_range.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "$K" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
for r in 1 2 3; do
  echo "-- A (${A:-tree})"; YOLOSOD_LIB_AB=$A timeout -k 10 120 python -u scripts/bench_ops.py "$@" 2>&1 | grep " ms " || exit 1
  echo "-- B (${B:-tree})"; YOLOSOD_LIB_AB=$B timeout -k 10 120 python -u scripts/bench_ops.py "$@" 2>&1 | grep " ms " || exit 1
done
