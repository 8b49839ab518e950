#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
  for f in "" GELU MLPMFMA EXP WLOAD DW; do
    lib=""; [ -n "$f" ] && lib=ablib/lib_abl_$f.so
    echo "-- ${f:-baseline}"
    YOLOSOD_LIB_AB=$lib timeout -k 10 120 python -u scripts/bench_ops.py swin_L28 2>&1 | grep " ms " || exit 1
  done
done
