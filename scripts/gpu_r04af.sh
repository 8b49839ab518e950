#!/bin/bash
# round 4: SE apply with 2 / 4 pixel quads per thread vs 1, and the unfused gate (same box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for v in 1 2 4; do echo "ppt $v"; YOLOSOD_SE_PPT=$v timeout -k 10 120 python3 scripts/bench_ops.py se_L1 se_L23 2>&1 | grep " ms "; done
  echo "unfused"; YOLOSOD_FUSED_GATES=0 timeout -k 10 120 python3 scripts/bench_ops.py se_L1 se_L23 2>&1 | grep " ms "
done
