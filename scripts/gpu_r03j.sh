#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
  for lib in "" ablib/lib_abl_HALO.so ablib/lib_abl_WLOAD.so; do
    echo "-- ${lib:-current}"
    YOLOSOD_LIB_AB=$lib timeout -k 10 120 python -u scripts/bench_ops.py swin_L28 swin_L9 2>&1 | grep " ms " || exit 1
  done
done
