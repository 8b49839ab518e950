#!/bin/bash
# GPU tests of the A2 / GEMM paths on the in-tree build, then same-box A/B against ab_push/lib_prev.so
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-a2ab}; mkdir -p $OUT
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  echo "-- prev"; YOLOSOD_LIB_AB=ab_push/lib_prev.so timeout -k 10 120 python -u scripts/bench_ops.py a2_L12 ${CASES} 2>&1 | grep " ms " || exit 1
  echo "-- tree"; timeout -k 10 120 python -u scripts/bench_ops.py a2_L12 ${CASES} 2>&1 | grep " ms " || exit 1
done
