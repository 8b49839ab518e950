#!/bin/bash
# round 4: Detect head weight prologue with unconditional loads: head tests, same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04aw}; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/yolo-sod_amd/lib_ab/libyolosod_hip_base.so
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_model.py tests/test_gpu_e2e.py tests/test_gpu_bf16.py tests/test_gpu_map.py -k "head or decode or e2e or map or model or predictor" > $O/pytest.log 2>&1 \
  || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  echo "base rep $rep"; YOLOSOD_LIB_AB=$BASE timeout -k 10 120 python3 scripts/bench_ops.py head 2>&1 | grep " ms "
  echo "new rep $rep"; timeout -k 10 120 python3 scripts/bench_ops.py head 2>&1 | grep " ms "
done
