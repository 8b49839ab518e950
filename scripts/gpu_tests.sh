#!/bin/bash
# GPU pytest pass only: bash scripts/gpu_tests.sh TAG [pytest -k expr] [test path]
set -o pipefail
TAG=${1:-run}
K=${2:-}
P=${3:-tests}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 900 python -u -m pytest $P -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "${KARG[@]}" > "$OUT/pytest.log" 2>&1
rc=$?
tail -40 "$OUT/pytest.log" | grep -E "FAILED|ERROR|passed|failed|Error" | tail -25
exit $rc
