#!/bin/bash
# bf16 GPU tests on the in-tree build, then same-box A/B of the bf16 GEMM (scripts/bench_gemm.py --bf16) and Swin
# L9_m / A2_m (bench_ops) against ab_push/lib_prev.so
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-gemmab}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "-- prev"; YOLOSOD_LIB_AB=ab_push/lib_prev.so timeout -k 10 120 python -u scripts/bench_gemm.py --bf16 --no-torch 2>&1 | grep " ms " || exit 1
  echo "-- tree"; timeout -k 10 120 python -u scripts/bench_gemm.py --bf16 --no-torch 2>&1 | grep " ms " || exit 1
done
for r in 1 2; do
  echo "-- prev"; YOLOSOD_LIB_AB=ab_push/lib_prev.so timeout -k 10 120 python -u scripts/bench_ops.py --bf16 swin_L9_m a2_L12_m 2>&1 | grep " ms " || exit 1
  echo "-- tree"; timeout -k 10 120 python -u scripts/bench_ops.py --bf16 swin_L9_m a2_L12_m 2>&1 | grep " ms " || exit 1
done
