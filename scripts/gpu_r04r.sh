#!/bin/bash
# round 4: same-box A/B of the channel-gate changes inside the bench (n640 only): per-op event ms + step time
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04r}; mkdir -p $O
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 240 python3 -u bench.py --no-cpu-baseline --no-nms-load --no-extra-configs --steps 20 \
    > $O/$name.json 2> $O/$name.err || { tail -5 $O/$name.err; exit 1; }
  python3 - $O/$name.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ops = {f"{o['op']}{o['shape'][1]}x{o['shape'][2]}": o['avg_ms'] for o in d['hip_ops']}
keep = ["se32x320", "cbam64x160", "ca128x80", "cbam256x40", "se128x80", "nms10x34000"]
print(f"{sys.argv[2]:10s} {d['value']:8.1f} img/s {d['ms_per_step']:7.3f} ms path {d['path_roofline']['frac']:.4f} "
      + " ".join(f"{k}={ops.get(k, float('nan')):.4f}" for k in keep))
PY
}
for rep in 1 2; do
  run def_$rep A=1
  run ca0_$rep YOLOSOD_CA_APPLY2=0
  run ps0_$rep YOLOSOD_CBAM_PS2=0
  run sep0_$rep YOLOSOD_SE_PRE=0
  run st0_$rep YOLOSOD_STREAMS=0
done
echo done
