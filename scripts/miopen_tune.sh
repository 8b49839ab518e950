#!/bin/bash
# MIOpen auto-tuning of the n640 backbone convs (MIOPEN_FIND_ENFORCE=SEARCH_DB_UPDATE: tunable solvers search their
# parameters, results into the user perf-db / find-db under gpurun_out/miotune/db), bounded to ~16 minutes.
set -o pipefail
OUT=gpurun_out/miotune; mkdir -p $OUT/db
cp yolo-sod_amd/miopen_db/*.ufdb.txt $OUT/db/ 2>/dev/null
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export MIOPEN_USER_DB_PATH="$GRAFT_REPO_ROOT/$OUT/db"
( while sleep 60; do ls -la $OUT/db | tail -4; done ) &
mon=$!
MIOPEN_FIND_MODE=NORMAL MIOPEN_FIND_ENFORCE=SEARCH_DB_UPDATE timeout -k 10 960 python3 -u bench.py --no-cpu-baseline \
  --no-nms-load --no-extra-configs --steps 2 --warmup 1 > $OUT/tune.json 2> $OUT/tune.err
rc=$?
kill $mon
echo "tune rc=$rc"; tail -3 $OUT/tune.err; ls -la $OUT/db
