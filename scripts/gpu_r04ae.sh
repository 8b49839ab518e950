#!/bin/bash
# round 4: SQ counters of the A2 kernels (proj / pool, qkv / attention, out GEMM)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04ae}; mkdir -p $O
bash scripts/sq_run.sh $O/sq a2_L12 > /dev/null && python3 scripts/sq_summary.py $O/sq
