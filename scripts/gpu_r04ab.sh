#!/bin/bash
# round 4: bf16 fused Swin (C=128) with swizzled T / U / QK tiles: tests, same-box A/B against the base library, SQ
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04ab}; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/yolo-sod_amd/lib_ab/libyolosod_hip_base.so
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_bf16.py > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  echo "base rep $rep"; YOLOSOD_LIB_AB=$BASE timeout -k 10 120 python3 scripts/bench_ops.py --bf16 swin_L28_m 2>&1 | grep " ms "
  echo "new rep $rep"; timeout -k 10 120 python3 scripts/bench_ops.py --bf16 swin_L28_m 2>&1 | grep " ms "
done
SQ_ARGS=--bf16 bash scripts/sq_run.sh $O/sq swin_L28_m > /dev/null && python3 scripts/sq_summary.py $O/sq | grep -A2 "swin_fused"
