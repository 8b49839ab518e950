#!/bin/bash
# Swin GPU tests + same-box A/B of the fp16-split kernels (default) against the exact-fp32-MFMA ones:
# bash scripts/ab_x3.sh TAG [bench_ops cases...]
set -o pipefail
TAG=${1:-x3}; shift
CASES=${@:-swin_L28 swin_L9}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "swin" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2; do
  echo "-- fp32 MFMA"; YOLOSOD_SWIN_X3=0 timeout -k 10 120 python -u scripts/bench_ops.py $CASES 2>&1 | grep " ms " || exit 1
  echo "-- f16x2"; timeout -k 10 120 python -u scripts/bench_ops.py $CASES 2>&1 | grep " ms " || exit 1
done
