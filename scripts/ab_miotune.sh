#!/bin/bash
# Same-box A/B of the committed MIOpen find-db against the auto-tuned one (find-db + perf-db from
# scripts/miopen_tune.sh, staged under ab_push/miodb_tuned): n640 bench, alternating, 3 runs each.
set -o pipefail
OUT=gpurun_out/abmio; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
A="$GRAFT_REPO_ROOT/yolo-sod_amd/miopen_db"; B="$GRAFT_REPO_ROOT/ab_push/miodb_tuned"
for i in 1 2 3; do
  for v in A B; do
    d=$A; [ $v = B ] && d=$B
    MIOPEN_USER_DB_PATH=$d timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-nms-load --no-extra-configs \
      --steps 30 --warmup 10 > $OUT/$v$i.json 2> $OUT/$v$i.err || { echo "fail $v$i"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$v$i.json'));print('$v$i',d['value'],d['ms_per_step'])"
  done
done
