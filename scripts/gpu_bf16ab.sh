#!/bin/bash
# bf16 GPU tests on the in-tree build, then same-box A/B against ab_push/lib_prev.so on bf16 bench_ops cases
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-bf16ab}; shift; mkdir -p $OUT
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "-- prev"; YOLOSOD_LIB_AB=ab_push/lib_prev.so timeout -k 10 120 python -u scripts/bench_ops.py --bf16 "$@" 2>&1 | grep " ms " || exit 1
  echo "-- tree"; timeout -k 10 120 python -u scripts/bench_ops.py --bf16 "$@" 2>&1 | grep " ms " || exit 1
done
bash scripts/prof_ops.sh ${OUT#gpurun_out/}_prof --bf16 swin_L9_m
