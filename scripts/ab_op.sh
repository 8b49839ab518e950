#!/bin/bash
# GPU tests (pytest -k EXPR over test_gpu_ops.py) + same-box A/B of an env toggle on bench_ops cases:
# bash scripts/ab_op.sh TAG "pytest -k expr" VAR VALUE_A VALUE_B case [case ...]
set -o pipefail
TAG=$1; K=$2; VAR=$3; VA=$4; VB=$5; shift 5
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "$K" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
for r in 1 2; do
  echo "-- $VAR=$VA"; env "$VAR=$VA" timeout -k 10 120 python -u scripts/bench_ops.py "$@" 2>&1 | grep " ms " || exit 1
  echo "-- $VAR=$VB"; env "$VAR=$VB" timeout -k 10 120 python -u scripts/bench_ops.py "$@" 2>&1 | grep " ms " || exit 1
done
