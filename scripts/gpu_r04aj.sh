#!/bin/bash
# round 4: SQ counters of the bf16 decomposed SwinBlock (L9_m: GEMMs, tokens + LN, window attention)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04aj}; mkdir -p $O
SQ_ARGS=--bf16 bash scripts/sq_run.sh $O/sq swin_L9_m > /dev/null && python3 scripts/sq_summary.py $O/sq
