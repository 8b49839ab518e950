#!/bin/bash
# round 4: thin 1x1 conv with the next x tile prefetched in registers: tests, in-model same-box A/B

set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04at}; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/yolo-sod_amd/lib_ab/libyolosod_hip_base.so
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_bf16.py -k "thin or cbam or model or conv" > $O/pytest.log 2>&1 \
  || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then export YOLOSOD_LIB_AB=$BASE; else unset YOLOSOD_LIB_AB; fi
    timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-extra-configs --no-nms-load > $O/bench_$lib.json 2> $O/bench_$lib.err || { tail -5 $O/bench_$lib.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1])
ca=[o for o in d['hip_ops'] if o['op']=='cbam'][0]
print('$lib', d['value'], d['path_roofline']['frac'], 'cbam', ca['avg_ms'], ca.get('producer_extra_ms'), ca.get('kernels_ms'))"
  done
done
