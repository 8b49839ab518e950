#!/bin/bash
# round 4: NMS prep with the class scores loaded before the in-place box stores: NMS / e2e tests, same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04ar}; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/yolo-sod_amd/lib_ab/libyolosod_hip_base.so
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_nms.py tests/test_gpu_e2e.py > $O/pytest.log 2>&1 \
  || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  echo "base rep $rep"; YOLOSOD_LIB_AB=$BASE timeout -k 10 200 python3 scripts/bench_nms.py 2>&1 | grep -E "^(predict|val) +(0|1000) "
  echo "new rep $rep"; timeout -k 10 200 python3 scripts/bench_nms.py 2>&1 | grep -E "^(predict|val) +(0|1000) "
done
