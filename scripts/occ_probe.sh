#!/bin/bash
# C = 64 Swin kernel at 3 / 2 / 1 workgroups per CU (LDS padding builds in ab_push/): how latency-bound it is
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
  for lib in "" ab_push/lib_pad10000.so ab_push/lib_pad40000.so; do
    echo "-- ${lib:-tree}"; YOLOSOD_LIB_AB=$lib timeout -k 10 120 python -u scripts/bench_ops.py swin_L28 2>&1 | grep " ms " || exit 1
  done
done
