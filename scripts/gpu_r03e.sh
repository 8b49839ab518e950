#!/bin/bash
set -o pipefail
TAG=${1:-r03e}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py -m gpu -q -k "gemm_bf16 or m_scale or transformer" --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for m in 3 2 0; do
  echo "-- GEMMB_GLDS=$m"
  YOLOSOD_GEMMB_GLDS=$m timeout -k 10 120 python -u scripts/bench_gemm.py --bf16 2>&1 | grep "M=" || exit 1
done
for m in 3 0; do
  echo "-- ops GEMMB_GLDS=$m"
  YOLOSOD_GEMMB_GLDS=$m timeout -k 10 120 python -u scripts/bench_ops.py --bf16 swin_L9_m a2_L12_m 2>&1 | grep " ms " || exit 1
done
exit $rc
