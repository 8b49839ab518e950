#!/bin/bash
# round 4: A2 proj / pool kernel in area groups (two 4-wave workgroups per CU): tests, same-box A/B, kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04ac}; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/yolo-sod_amd/lib_ab/libyolosod_hip_base.so
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_ops.py -k "a2" > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  echo "base rep $rep"; YOLOSOD_LIB_AB=$BASE timeout -k 10 120 python3 scripts/bench_ops.py a2_L12 2>&1 | grep " ms "
  echo "new rep $rep"; timeout -k 10 120 python3 scripts/bench_ops.py a2_L12 2>&1 | grep " ms "
done
for px in 400 100; do
  echo "cap $px"; YOLOSOD_A2_POOL_PX=$px timeout -k 10 120 python3 scripts/bench_ops.py a2_L12 2>&1 | grep " ms "
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- python3 scripts/bench_ops.py a2_L12 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
f=$(find $O/kt -name "kt_kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -12
