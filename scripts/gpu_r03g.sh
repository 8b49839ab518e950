#!/bin/bash
set -o pipefail
TAG=${1:-r03g}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_split_range.py -m gpu -q -k "swin or split" --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -12
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for lib in "" ablib/lib_abl_X3_PRIO.so; do
    echo "-- ${lib:-current}"
    YOLOSOD_LIB_AB=$lib timeout -k 10 120 python -u scripts/bench_ops.py swin_L28 2>&1 | grep " ms " || exit 1
  done
done
