#!/bin/bash
# Same-box A/B of the default bench (n640 only, no CPU baseline / NMS load) under two environments:
#   bash scripts/gpu_benchab.sh TAG "ENV_A" "ENV_B" [reps]   e.g. "YOLOSOD_SIDE_STREAMS=1" "YOLOSOD_SIDE_STREAMS=3"
set -o pipefail
TAG=$1; EA=$2; EB=$3; R=${4:-2}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in $(seq 1 $R); do
  for V in A B; do
    if [ $V = A ]; then E=$EA; else E=$EB; fi
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-nms-load --no-extra-configs \
      --detail-json "$OUT/detail_${V}_$r.json" > "$OUT/bench_${V}_$r.json" 2> "$OUT/err_${V}_$r.txt" || { tail -5 "$OUT/err_${V}_$r.txt"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_${V}_$r.json').read().strip().splitlines()[-1]); print('$V ($E)', d['value'], d['ms_per_step'], 'path', d['path_roofline']['frac'], {k: v for k, v in d['hip_ops_avg_ms'].items() if k.startswith(('swin','ca','a2','se:32x32'))})"
  done
done
