#!/bin/bash
# round 4: branch-free tile loads (A2 proj / pool, fp32 / bf16 GEMMs), A2 area groups: tests, same-box A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-r04ad}; mkdir -p $O
BASE=$GRAFT_REPO_ROOT/yolo-sod_amd/lib_ab/libyolosod_hip_base.so
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ops.py tests/test_gpu_bf16.py \
  tests/test_gpu_split_range.py > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for rep in 1 2; do
  echo "base rep $rep"; YOLOSOD_LIB_AB=$BASE timeout -k 10 180 python3 scripts/bench_ops.py a2_L12 a2_L12_1280 2>&1 | grep " ms "
  YOLOSOD_LIB_AB=$BASE timeout -k 10 180 python3 scripts/bench_ops.py --bf16 swin_L9_m a2_L12_m 2>&1 | grep " ms "
  echo "new rep $rep"; timeout -k 10 180 python3 scripts/bench_ops.py a2_L12 a2_L12_1280 2>&1 | grep " ms "
  timeout -k 10 180 python3 scripts/bench_ops.py --bf16 swin_L9_m a2_L12_m 2>&1 | grep " ms "
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o kt -- python3 scripts/bench_ops.py a2_L12 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/ktm -o kt -- python3 scripts/bench_ops.py --bf16 swin_L9_m > $O/ktm.log 2>&1 || { tail -5 $O/ktm.log; exit 1; }
for d in kt ktm; do f=$(find $O/$d -name "kt_kernel_stats.csv" | head -1); python3 -c "
import csv
for r in list(csv.DictReader(open('$f')))[:8]: print(r['Name'][:70], r['Calls'], r['AverageNs'])"; done
