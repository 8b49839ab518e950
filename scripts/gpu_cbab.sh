#!/bin/bash
# channel-attention GPU tests on the in-tree build + same-box A/B (fp32 and bf16 cases) against ab_push/lib_prev.so
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-cbab}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_bf16.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "-- prev"; YOLOSOD_LIB_AB=ab_push/lib_prev.so timeout -k 10 120 python -u scripts/bench_ops.py cbam_L4 cbam_L18 ca_L32 2>&1 | grep " ms " || exit 1
  YOLOSOD_LIB_AB=ab_push/lib_prev.so timeout -k 10 120 python -u scripts/bench_ops.py --bf16 cbam_L4_m ca_L32_m 2>&1 | grep " ms " || exit 1
  echo "-- tree"; timeout -k 10 120 python -u scripts/bench_ops.py cbam_L4 cbam_L18 ca_L32 2>&1 | grep " ms " || exit 1
  timeout -k 10 120 python -u scripts/bench_ops.py --bf16 cbam_L4_m ca_L32_m 2>&1 | grep " ms " || exit 1
done
