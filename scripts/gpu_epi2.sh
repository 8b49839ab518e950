#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/epi2
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/epi2/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/epi2/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "-- prev"; YOLOSOD_LIB_AB=ab_push/lib_prev.so timeout -k 10 120 python -u scripts/bench_epi.py --bf16 || exit 1
  echo "-- tree"; timeout -k 10 120 python -u scripts/bench_epi.py --bf16 || exit 1
done
