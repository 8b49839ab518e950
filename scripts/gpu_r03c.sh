#!/bin/bash
set -o pipefail
TAG=${1:-r03c}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 400 python -u -m pytest tests/test_gpu_split_range.py tests/test_gpu_e2e.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/sq_run.sh "$OUT/sq" swin_L28 swin_L9 || exit 1
YOLOSOD_LIB_AB=ablib/lib_diag.so timeout -k 10 120 python -u scripts/diag_x3.py > "$OUT/diag_x3.txt" 2>&1 || exit 1
YOLOSOD_LIB_AB=ablib/lib_diag.so timeout -k 10 120 python -u scripts/diag_wx.py > "$OUT/diag_wx.txt" 2>&1 || exit 1
cat "$OUT/diag_x3.txt" "$OUT/diag_wx.txt"
exit $rc
