#!/bin/bash
# round 4: full suite + profiled bench with its per-launch CSV (recompute check) + the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04s}
TAG=${TAG:-r04s} bash scripts/gpu_r04o.sh || exit 1
timeout -k 10 500 python3 -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['path_roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))
print(d['nms_loaded'])
for k, c in d.get('configs', {}).items(): print(k, c['value'], c['path_roofline']['frac'])
"
