#!/bin/bash
# same-box A/B of diagnostic library builds on the Swin cases
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
  for lib in "" ablib/lib_occ2.so ablib/lib_ps80.so; do
    echo "-- lib ${lib:-current}"
    YOLOSOD_LIB_AB=$lib timeout -k 10 120 python -u scripts/bench_ops.py swin_L28 2>&1 | grep " ms " || exit 1
  done
done
