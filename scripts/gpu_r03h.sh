#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for lib in ""; do
  echo "-- ${lib:-current}"
  YOLOSOD_LIB_AB=$lib timeout -k 10 120 python -u scripts/check_swin.py swin_L28 2>&1 | grep "max|err|" || exit 1
done
