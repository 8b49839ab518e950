#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_round.sh r03y n640 || exit 1
for r in 1 2; do
  echo "-- prev"; YOLOSOD_LIB_AB=ab_push/lib_prev.so timeout -k 10 120 python -u scripts/bench_ops.py se_L1 se_L23 2>&1 | grep " ms " || exit 1
  echo "-- tree"; timeout -k 10 120 python -u scripts/bench_ops.py se_L1 se_L23 2>&1 | grep " ms " || exit 1
done
bash scripts/prof_cfg.sh r03y m640
