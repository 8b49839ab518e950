#!/bin/bash
# round 4: channel-attention / A2 / GEMM GPU tests, then the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04ag}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_bf16.py > $O/pytest.log 2>&1 \
  || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python3 -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['path_roofline']['frac'])
for o in d['hip_ops']: print(' ', o['op'], o['shape'], o['avg_ms'], o['frac'], o.get('producer_extra_ms'))
for k, c in d.get('configs', {}).items(): print(k, c['value'], c['path_roofline']['frac'])
"
