#!/bin/bash
# C = 64 Swin kernel: stage stamps and ablation timings (ab_push/ holds the diagnostic builds)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r03k
YOLOSOD_LIB_AB=ab_push/lib_diag.so timeout -k 10 120 python -u scripts/diag_x3.py > gpurun_out/r03k/diag_x3.txt 2>&1 || exit 1
cat gpurun_out/r03k/diag_x3.txt
for r in 1 2; do
  for f in "" WLOAD HALO GELU MLPMFMA; do
    lib=""; [ -n "$f" ] && lib=ab_push/lib_abl_$f.so
    echo "-- ${f:-baseline}"
    YOLOSOD_LIB_AB=$lib timeout -k 10 120 python -u scripts/bench_ops.py swin_L28 2>&1 | grep " ms " || exit 1
  done
done
