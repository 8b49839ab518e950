#!/bin/bash
# Selected GPU tests: bash scripts/gpu_tests.sh TAG test_file[::name] ...  (results under gpurun_out/TAG)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export YOLOSOD_PARITY_LOG="$GRAFT_REPO_ROOT/$OUT/parity.log"
timeout -k 10 900 python -u -m pytest "$@" -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -40
exit $rc
