#!/bin/bash
# round 4: kernel trace of the C=64 Swin split pair vs the one-kernel form
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
YOLOSOD_SWIN_SPLIT=1 bash scripts/prof_ops.sh r04b_split swin_L28 || exit 1
YOLOSOD_SWIN_SPLIT=0 bash scripts/prof_ops.sh r04b_one swin_L28 || exit 1
