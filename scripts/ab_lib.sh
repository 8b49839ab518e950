#!/bin/bash
# GPU tests (pytest -k EXPR over the op test files) + same-box A/B of a diagnostic library build against the current
# one on bench_ops cases: bash scripts/ab_lib.sh TAG "pytest -k expr" LIB_A [--bf16] case [case ...]
set -o pipefail
TAG=$1; K=$2; A=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "$K" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
for r in 1 2; do
  echo "-- A ($A)"; YOLOSOD_LIB_AB=$A timeout -k 10 120 python -u scripts/bench_ops.py "$@" 2>&1 | grep " ms " || exit 1
  echo "-- B (current)"; timeout -k 10 120 python -u scripts/bench_ops.py "$@" 2>&1 | grep " ms " || exit 1
done
