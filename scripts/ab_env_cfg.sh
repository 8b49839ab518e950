#!/bin/bash
# Same-box A/B of an environment toggle on one bench config: bash scripts/ab_env_cfg.sh TAG CONFIG VAR VALUE_A VALUE_B
set -o pipefail
TAG=$1; CFG=$2; VAR=$3; VA=$4; VB=$5
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in 1 2; do
  env "$VAR=$VA" timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline --no-nms-load > "$OUT/a$i.json" 2> "$OUT/a$i.err" || exit 1
  env "$VAR=$VB" timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline --no-nms-load > "$OUT/b$i.json" 2> "$OUT/b$i.err" || exit 1
done
python - "$OUT" <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f))
    ops = {f"{o['op']}{o['shape'][1]}": o["avg_ms"] for o in d["hip_ops"]}
    print(os.path.basename(f), d["value"], d["ms_per_step"], d["path_roofline"]["frac"], ops)
PY
