#!/bin/bash
# round 4: Swin C=256 swizzled planes: tests, same-box bench_ops A/B against the saved base library, SQ counters
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04x}; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/yolo-sod_amd/lib_ab/libyolosod_hip_base.so
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_split_range.py \
  tests/test_gpu_model.py -k "swin or L9 or model" > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  echo "base rep $rep"; YOLOSOD_LIB_AB=$BASE timeout -k 10 120 python3 scripts/bench_ops.py swin_L9 swin_L9_1280 swin_L28 2>&1 | grep " ms "
  echo "new rep $rep"; timeout -k 10 120 python3 scripts/bench_ops.py swin_L9 swin_L9_1280 swin_L28 2>&1 | grep " ms "
done
bash scripts/sq_run.sh $O/sq swin_L9 > /dev/null && python3 scripts/sq_summary.py $O/sq | grep -A2 "swin_wx"
