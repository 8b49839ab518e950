#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/epi
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/epi/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/epi/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  echo "-- prev"; YOLOSOD_LIB_AB=ab_push/lib_prev.so timeout -k 10 120 python -u scripts/bench_epi.py || exit 1
  echo "-- tree"; timeout -k 10 120 python -u scripts/bench_epi.py || exit 1
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-nms-load --no-extra-configs > gpurun_out/epi/bench.json 2> gpurun_out/epi/bench.err || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/epi/bench.json | head -1
