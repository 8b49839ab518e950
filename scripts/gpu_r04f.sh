#!/bin/bash
# round 4: GPU suite from the e2e test on (parity log) + default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04f; mkdir -p $O
export YOLOSOD_PARITY_LOG=$O/parity_margins.txt
timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_e2e.py tests/test_gpu_map.py tests/test_gpu_model.py tests/test_gpu_nms.py tests/test_gpu_ops.py tests/test_gpu_split_range.py tests/test_gpu_upsample.py > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/pytest.log | head -30; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['path_roofline'])
for o in d['hip_ops']: print(o['op'], o['shape'], o['avg_ms'], o['frac'])
for k, c in d.get('configs', {}).items(): print(k, c['value'], c['path_roofline']['frac'])
"
exit $rc
