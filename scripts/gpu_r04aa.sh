#!/bin/bash
# round 4: head / e2e / map tests + default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04aa}; mkdir -p $O
export YOLOSOD_PARITY_LOG=$O/parity_margins.txt
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_e2e.py \
  tests/test_gpu_map.py tests/test_gpu_model.py tests/test_gpu_checkpoint.py -k "head or e2e or map or model or checkpoint or decode" > $O/pytest.log 2>&1 \
  || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 scripts/bench_ops.py head 2>&1 | grep " ms "
timeout -k 10 500 python3 -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['path_roofline']['frac'])
for o in d['hip_ops']: print(' ', o['op'], o['shape'], o['avg_ms'], o['frac'])
for k, c in d.get('configs', {}).items(): print(k, c['value'], c['path_roofline']['frac'])
"
