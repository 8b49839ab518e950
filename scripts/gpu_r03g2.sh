#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r03g
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/gpurun_out/r03g/parity.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_split_range.py tests/test_gpu_model.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r03g/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03g/pytest.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "-- prev"; YOLOSOD_LIB_AB=ab_push/lib_prev.so timeout -k 10 120 python -u scripts/bench_ops.py a2_L12 2>&1 | grep " ms " || exit 1
  echo "-- tree"; timeout -k 10 120 python -u scripts/bench_ops.py a2_L12 2>&1 | grep " ms " || exit 1
done
bash scripts/occ_probe.sh
